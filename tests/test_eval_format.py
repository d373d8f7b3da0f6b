"""OpenFHE EVALUATION-format key ingest (tfhe_setup_eval).

OpenFHE keeps the bootstrapping key in EVALUATION format: the negacyclic NTT with
root RootOfUnity(2N, Q) (the smallest primitive 2N-th root, nbtheory.cpp:284-343) and
bit-reversed output (transformnat-impl.h:196-236, 684-706).  The CPU tests pin the
oracle's restatement of that format two independent ways: the root against a
brute-force search written here, and the transform against direct polynomial
evaluation (output i = a(root^(2 bitrev(i) + 1))).  No reference-run fixture holds
EVALUATION-format values, so the format itself is restated from source, not pinned by
reference output.  The GPU tests check that keys ingested in that format give exactly the
outputs of coefficient-format ingest (and of the oracle) on every kernel family.
"""
import numpy as np
import pytest

SETS = ["TOY", "MEDIUM", "STD128", "STD192", "STD128Q", "STD256"]


def _bitrev(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2)


def _min_primitive_root(Q, N):
    # any primitive 2N-th root r (r^N = -1), then the minimum over r^k, k odd < 2N
    g = 2
    while True:
        r = pow(g, (Q - 1) // (2 * N), Q)
        if pow(r, N, Q) == Q - 1:
            break
        g += 1
    return min(pow(r, k, Q) for k in range(1, 2 * N, 2))


@pytest.mark.parametrize("name", SETS)
def test_root_of_unity_is_minimal_primitive(oracle, name):
    p = oracle.params_from_set(name)
    assert oracle.root_of_unity(p.Q, p.N) == _min_primitive_root(p.Q, p.N)


def test_root_of_unity_logq_context(oracle):
    p = oracle.params_from_logq("STD128", True, 12, 0, 0, 1)  # Q = 2^54 - 77823, N = 2048
    r = oracle.root_of_unity(p.Q, p.N)
    assert r == _min_primitive_root(p.Q, p.N)
    assert pow(r, p.N, p.Q) == p.Q - 1


@pytest.mark.parametrize("name", ["STD128", "STD192"])
def test_openfhe_ntt_is_bitreversed_evaluation(oracle, name):
    p = oracle.params_from_set(name)
    Q, N = p.Q, p.N
    logN = N.bit_length() - 1
    rs = np.random.default_rng(3)
    a = rs.integers(0, Q, N, dtype=np.uint64)
    ev = oracle.openfhe_ntt(Q, N, a)
    psi = oracle.root_of_unity(Q, N)
    coeffs = [int(v) for v in a]
    for i in (0, 1, 2, 5, N // 2, N - 1):
        x = pow(psi, 2 * _bitrev(i, logN) + 1, Q)
        acc = 0
        for c in reversed(coeffs):  # Horner
            acc = (acc * x + c) % Q
        assert int(ev[i]) == acc, i
    assert np.array_equal(oracle.openfhe_ntt(Q, N, ev, inverse=True), a)


# ---------------------------------------------------------------- GPU
def _ctxs(capi, oracle, cp, op, bsk, ksk, env=None):
    import os

    ev = oracle.openfhe_ntt(op.Q, op.N, bsk)
    if env:
        os.environ[env] = "1"
    try:
        c1 = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
        c2 = capi.BinFHEContextHIP(cp).GPUSetup(ev, ksk, bsk_format="evaluation")
    finally:
        if env:
            os.environ.pop(env, None)
    return c1, c2, ev


@pytest.mark.gpu
@pytest.mark.parametrize("pset,env", [("STD128", None), ("STD128", "TFHE_FORCE_GENERIC"), ("STD192", None)])
def test_eval_format_ingest_matches_coefficient_ingest(oracle, pset, env):
    import tfhe_amd as capi

    op = oracle.params_from_set(pset)
    cp = capi.params_from_set(pset)
    sk, bsk, ksk = oracle.keygen(op, oracle.Rng(11))
    c1, c2, _ = _ctxs(capi, oracle, cp, op, bsk, ksk, env)
    orc = oracle.Oracle(op, bsk, ksk)
    rs = np.random.default_rng(5)
    B = 6
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    g1, g2 = c1.EvalAcc(a, op.q, acc), c2.EvalAcc(a, op.q, acc)
    assert np.array_equal(g1, g2)
    assert np.array_equal(g2, orc.eval_acc(a, op.q, acc))
    bits = rs.integers(0, 2, (2, B))
    ct1 = np.stack([oracle.encrypt(op, oracle.Rng(100 + i), sk, int(bits[0, i]), 4, op.q) for i in range(B)])
    ct2 = np.stack([oracle.encrypt(op, oracle.Rng(200 + i), sk, int(bits[1, i]), 4, op.q) for i in range(B)])
    out = c2.EvalBinGate("NAND", ct1, ct2)
    assert np.array_equal(out, c1.EvalBinGate("NAND", ct1, ct2))
    for i in range(B):
        assert oracle.decrypt(op, sk, out[i], 4, op.q) == 1 - (bits[0, i] & bits[1, i])
    c1.GPUClean(), c2.GPUClean(), orc.close()


@pytest.mark.gpu
def test_eval_format_logq_context(oracle):
    """54-bit Q (generic u64 kernel): evaluation-format ingest, EvalFunc parity."""
    import tfhe_amd as capi

    from helpers import cube_lut

    op = oracle.params_from_logq("STD128", True, 12, 0, 0, 1)
    cp = capi.params_from_logq("STD128", True, 12, 0, 0, 1)
    sk, bsk, ksk = oracle.keygen(op, oracle.Rng(12))
    c1, c2, _ = _ctxs(capi, oracle, cp, op, bsk, ksk)
    ct = np.stack([oracle.encrypt(op, oracle.Rng(300 + i), sk, i % 8, 8, op.q) for i in range(4)])
    lut = cube_lut(op.q)
    assert np.array_equal(c1.EvalFunc(ct, lut), c2.EvalFunc(ct, lut))
    c1.GPUClean(), c2.GPUClean()


@pytest.mark.gpu
def test_eval_format_rejects_unreduced_entries(oracle):
    import tfhe_amd as capi

    op = oracle.params_from_set("STD128")
    cp = capi.params_from_set("STD128")
    _, bsk, ksk = oracle.keygen(op, oracle.Rng(13))
    ev = oracle.openfhe_ntt(op.Q, op.N, bsk)
    ev[12345] = op.Q
    with pytest.raises(capi.TfheError):
        capi.BinFHEContextHIP(cp).GPUSetup(ev, ksk, bsk_format="evaluation")
