"""GPU: BASELINE configurations at their full batch inside the -m gpu suite (verdict r3, weak 1):
  * C3 -- EvalFunc(x^3 mod 8) on the arbFunc logQ = 12 context (sf2, one digit), B = 4096, the cube
    LUT of GenerateLUTviaFunction; sampled ciphertexts on both ends and in the middle equal the oracle;
  * C4 -- STD192 NAND (f64w) across the 65,536-ciphertext device chunk (the reference's
    max_bootstapping_num), B = 65,539; samples on both sides of the boundary equal the oracle.
Keys: Appendix B splitmix64 keys (tests/helpers.kat_inputs' generator); inputs: seeded uniform
ciphertexts (parity, not decryption, is checked).
"""
import numpy as np
import pytest

from helpers import cube_lut, random_cts

pytestmark = pytest.mark.gpu


def test_c3_evalfunc_full_batch(shared_kat):
    s = shared_kat("ARB12")  # the session's shared context
    cp, ctx, orc = s["cp"], s["ctx"], s["orc"]
    assert ctx.info().br_kernel == 5  # special form
    rs = np.random.default_rng(3)
    B = 4096
    ct = random_cts(rs, B, cp.n, cp.q)
    lut = cube_lut(cp.q)
    out = ctx.EvalFunc(ct, lut)
    idx = [0, 1, 2047, 4094, 4095]
    assert np.array_equal(out[idx], orc.eval_func(ct[idx], lut, cp.q))


def test_c4_std192_across_the_chunk_boundary(shared_kat):
    s = shared_kat("STD192")  # the session's shared context
    cp, ctx, orc = s["cp"], s["ctx"], s["orc"]
    rs = np.random.default_rng(4)
    B = 65536 + 3
    c1 = random_cts(rs, B, cp.n, cp.q)
    c2 = random_cts(rs, B, cp.n, cp.q)
    out = ctx.EvalBinGate("NAND", c1, c2)
    idx = [0, 65535, 65536, B - 1]
    assert np.array_equal(out[idx], orc.eval_bin_gate("NAND", c1[idx], c2[idx]))
