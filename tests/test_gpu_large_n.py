"""GPU: ring dimensions past 2048.  GenerateBinFHEContext(set, arbFunc, logQ, N, ...) takes any larger
power-of-two N (binfhecontext.cpp:94-96) and the reference dispatches N/2 up to 4096 in its FFT kernel
(bootstrapping.cu:772-871).  Here N = 4096 / 8192 run on the generic register-resident kernel with
1024-thread workgroups (k_blind_rotate_gen2<W, CN, 1024>, blind_rotate_generic.hip) and the key switch
with one wavefront per workgroup when four digit arrays do not fit the LDS (N = 8192, lwe_kernels.hip).
TOY lattice (n = 32) to keep the keys small; valid keys from the oracle's keygen.  Checks: bit-exact
against the oracle (which tests/test_oracle_ref_vectors.py pins to the reference's own outputs at both
N: toy4096_funcvec, toy8192_sign) and decryption of every output.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def cube_lut(q, P):
    interval = q // P
    return np.array([((i // interval) ** 3 % P) * interval for i in range(q)], dtype=np.uint64)


@pytest.fixture(scope="module", params=[(1, 12, 4096), (0, 23, 8192)], ids=["arb12_N4096", "logQ23_N8192"])
def ctx(request, oracle):
    import tfhe_amd

    arb, logq, N = request.param
    op = oracle.params_from_logq("TOY", bool(arb), logq, N, 0, 1)
    cp = tfhe_amd.params_from_logq("TOY", bool(arb), logq, N, 0, 1)
    assert op.N == N and cp.N == N
    rng = oracle.Rng(44 + N)
    sk, bsk, ksk = oracle.keygen(op, rng)
    c = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    yield dict(op=op, sk=sk, ctx=c, orc=orc, rng=rng, arb=arb)
    c.GPUClean()
    orc.close()


def test_large_n_gate_matches_oracle_and_decrypts(ctx, oracle):
    op, sk, c, orc, rng = ctx["op"], ctx["sk"], ctx["ctx"], ctx["orc"], ctx["rng"]
    if ctx["arb"]:
        pytest.skip("gates need q = 2N (arbFunc contexts use q = N)")
    m1 = np.array([0, 0, 1, 1] * 4)
    m2 = np.array([0, 1, 0, 1] * 4)
    c1 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m1])
    c2 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m2])
    g = c.EvalBinGate("NAND", c1, c2)
    assert np.array_equal(g, orc.eval_bin_gate("NAND", c1, c2))
    assert [oracle.decrypt(op, sk, r, 4, op.q) for r in g] == [1 - (x & y) for x, y in zip(m1, m2)]


def test_large_n_func_or_sign(ctx, oracle):
    op, sk, c, orc, rng = ctx["op"], ctx["sk"], ctx["ctx"], ctx["orc"], ctx["rng"]
    if ctx["arb"]:  # EvalFunc, cube LUT over p = GetMaxPlaintextSpace (UnitTestFunc.cpp:44-68)
        P = c.GetMaxPlaintextSpace()
        lut = cube_lut(op.q, P)
        ms = np.arange(P)
        ct = np.stack([oracle.encrypt(op, rng, sk, int(m), P, op.q) for m in ms])
        out = c.EvalFunc(ct, lut)
        assert np.array_equal(out, orc.eval_func(ct, lut))
        assert [oracle.decrypt(op, sk, r, P, op.q) for r in out] == [int(m) ** 3 % P for m in ms]
    else:  # EvalSign, Qin = 2^23
        QIN = 1 << 23
        p = (op.q // 128 // 2) * (QIN // op.q)
        ms = np.array([0, 1, p // 4, p // 2 - p // 16, p // 2 + p // 16, 3 * p // 4, p - p // 16, p // 3])
        ct = np.stack([oracle.encrypt(op, rng, sk, int(m), p, QIN) for m in ms])
        out = c.EvalSign(ct, QIN)
        assert np.array_equal(out, orc.eval_sign(ct, QIN))
        assert [oracle.decrypt(op, sk, r, 2, op.q) for r in out] == [int(m >= p // 2) for m in ms]


@pytest.mark.parametrize("N,knob", [(2048, 0), (2048, 2), (4096, 0), (8192, 0)])
def test_u32_words_large_n_blind_rotation(oracle, N, knob):
    """logQ = 11 with N >= 2048 keeps a 27-bit Q (2 dG2 Q < 2^32): the generic kernels on u32 words --
    gen3<u32> at N = 2048 (v2 with the generic knob 2), v2 with 1024-thread workgroups at 4096 / 8192 --
    against the oracle, random keys and accumulators (TOY lattice)."""
    import tfhe_amd

    op = oracle.params_from_logq("TOY", False, 11, N, 0, 0)
    cp = tfhe_amd.params_from_logq("TOY", False, 11, N, 0, 0)
    rs = np.random.default_rng(N + knob)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    c = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    try:
        assert c.info().word_bits == 32 and c.info().br_kernel == 0
        c.set_knobs(generic=knob)
        a = rs.integers(0, op.q, (2, op.n), dtype=np.uint64)
        acc = rs.integers(0, op.Q, (2, 2, op.N), dtype=np.uint64)
        assert np.array_equal(c.EvalAcc(a, op.q, acc), orc.eval_acc(a, op.q, acc))
    finally:
        c.GPUClean()
        orc.close()
