"""Every BINFHE_PARAMSET (binfhe-constants.h:46-101, GenerateBinFHEContext tables at
binfhecontext.cpp:130-181) through the GPU with the GINX accumulator: bit-exact against the
oracle on random ciphertexts (uniform keys, the KAT recipe of SURVEY.md Appendix B), and,
for the smaller sets, decrypt-correct gates under valid keys (UnitTestFHEW.cpp's
assertions).  Covers every kernel the dispatcher can pick: fast (STD128 class), exact FP64
(STD192/STD128Q classes), generic v2 u32/u64 (N = 1024/2048) and generic v1 (TOY, N = 512).
"""
import numpy as np
import pytest

from helpers import random_cts

pytestmark = pytest.mark.gpu

ALL_SETS = ["TOY", "MEDIUM", "STD128_AP", "STD128_APOPT", "STD128", "STD128_OPT", "STD192", "STD192_OPT",
            "STD256", "STD256_OPT", "STD128Q", "STD128Q_OPT", "STD192Q", "STD192Q_OPT", "STD256Q", "STD256Q_OPT",
            "SIGNED_MOD_TEST"]
TRUTH = {"AND": lambda x, y: x & y, "OR": lambda x, y: x | y, "NAND": lambda x, y: 1 - (x & y),
         "NOR": lambda x, y: 1 - (x | y), "XOR": lambda x, y: x ^ y, "XNOR": lambda x, y: 1 - (x ^ y),
         "XOR_FAST": lambda x, y: x ^ y, "XNOR_FAST": lambda x, y: 1 - (x ^ y)}  # UnitTestFHEW.cpp truth tables


@pytest.mark.parametrize("name", ALL_SETS)
def test_paramset_gate_parity(oracle, name):
    import tfhe_amd as capi

    op = oracle.params_from_set(name)
    cp = capi.params_from_set(name)
    assert all(getattr(op, k) == getattr(cp, k) for k, _ in cp._fields_)
    bsk, ksk = oracle.kat_keys(op, oracle.Rng(21))
    ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    rs = np.random.default_rng(sum(name.encode()))
    c1 = random_cts(rs, 3, op.n, op.q)
    c2 = random_cts(rs, 3, op.n, op.q)
    assert np.array_equal(ctx.EvalBinGate("NAND", c1, c2), orc.eval_bin_gate("NAND", c1, c2))
    if op.N <= 1024:  # XOR = 3 bootstraps; the oracle's N = 2048 sets take seconds each
        assert np.array_equal(ctx.EvalBinGate("XOR", c1, c2), orc.eval_bin_gate("XOR", c1, c2))
    ctx.GPUClean()
    orc.close()


@pytest.mark.parametrize("name", ["TOY", "MEDIUM", "STD128_AP", "STD256", "STD192Q", "SIGNED_MOD_TEST"])
def test_paramset_gates_decrypt(oracle, name):
    import tfhe_amd as capi

    op = oracle.params_from_set(name)
    cp = capi.params_from_set(name)
    rng = oracle.Rng(31)
    sk, bsk, ksk = oracle.keygen(op, rng)
    ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    m1 = [0, 0, 1, 1]
    m2 = [0, 1, 0, 1]
    c1 = np.stack([oracle.encrypt(op, rng, sk, m, 4, op.q) for m in m1])
    c2 = np.stack([oracle.encrypt(op, rng, sk, m, 4, op.q) for m in m2])
    for gate, f in TRUTH.items():
        out = ctx.EvalBinGate(gate, c1, c2)
        assert [oracle.decrypt(op, sk, r, 4, op.q) for r in out] == [f(x, y) for x, y in zip(m1, m2)], gate
    ctx.GPUClean()
