"""Unit checks of the oracle's building blocks against independent restatements."""
import numpy as np
import pytest


def test_ntt_polymul_matches_schoolbook(oracle):
    for name in ("TOY", "STD128"):
        p = oracle.params_from_set(name)
        rs = np.random.default_rng(5)
        a = rs.integers(0, p.Q, p.N, dtype=np.uint64)
        b = rs.integers(0, p.Q, p.N, dtype=np.uint64)
        c1 = np.empty(p.N, dtype=np.uint64)
        c2 = np.empty(p.N, dtype=np.uint64)
        oracle.lib().or_polymul_schoolbook(__import__("ctypes").byref(p), a, b, c1)
        oracle.lib().or_polymul_ntt(__import__("ctypes").byref(p), a, b, c2)
        assert np.array_equal(c1, c2)


def test_roundqQ_matches_double_formula(oracle):
    import math

    rs = np.random.default_rng(1)
    for Q, q in [(134215681, 16384), (18014398509404161, 1 << 35), (1 << 35, 2048), (1 << 23, 1 << 21)]:
        for v in list(rs.integers(0, Q, 200)) + [0, Q - 1, Q // 2]:
            v = int(v)
            want = int(math.floor(0.5 + float(v) * float(q) / float(Q))) % q
            assert oracle.lib().or_roundqQ(v, q, Q) == want


def decompose_ref(p, poly):
    """Pure-Python restatement of rgsw-acc.cpp:80-110 (int64 arithmetic shifts)."""
    out = np.zeros((p.dG2, p.N), dtype=np.uint64)
    Q = p.Q
    lg = p.logG
    digits = p.digitsG - p.numDigitsToThrow
    for j in range(2):
        for k in range(p.N):
            t = int(poly[j, k])
            d = t if t < (Q >> 1) else t - Q
            for _ in range(p.numDigitsToThrow):
                r = ((d & ((1 << lg) - 1)) ^ (1 << (lg - 1))) - (1 << (lg - 1))
                d = (d - r) >> lg
            for l in range(digits):
                r = ((d & ((1 << lg) - 1)) ^ (1 << (lg - 1))) - (1 << (lg - 1))
                d = (d - r) >> lg
                out[j + 2 * l, k] = r + Q if r < 0 else r
    return out


@pytest.mark.parametrize("which", ["STD128", "arb12"])
def test_signed_digit_decompose(oracle, which):
    import ctypes

    p = oracle.params_from_set("STD128") if which == "STD128" else oracle.params_from_logq("STD128", True, 12, 0, 0, 1)
    p.N = 64  # decomposition is per coefficient; a short poly suffices
    rs = np.random.default_rng(3)
    poly = rs.integers(0, p.Q, (2, p.N), dtype=np.uint64)
    poly[0, :4] = [0, p.Q - 1, p.Q >> 1, (p.Q >> 1) + 1]
    out = np.empty((p.dG2, p.N), dtype=np.uint64)
    oracle.lib().or_signed_digit_decompose(ctypes.byref(p), poly.ravel(), out.ravel())
    assert np.array_equal(out, decompose_ref(p, poly))


def test_valid_keys_gates_decrypt(oracle):
    """Decrypt-correctness of every gate with the oracle's own valid keys (UnitTestFHEW.cpp:314-856 pattern)."""
    p = oracle.params_from_set("TOY")
    rng = oracle.Rng(11)
    sk, bsk, ksk = oracle.keygen(p, rng)
    o = oracle.Oracle(p, bsk, ksk)
    truth = {"AND": lambda x, y: x & y, "OR": lambda x, y: x | y, "NAND": lambda x, y: 1 - (x & y),
             "NOR": lambda x, y: 1 - (x | y), "XOR": lambda x, y: x ^ y, "XNOR": lambda x, y: 1 - (x ^ y),
             "XOR_FAST": lambda x, y: x ^ y, "XNOR_FAST": lambda x, y: 1 - (x ^ y)}
    m1 = np.array([0, 0, 1, 1])
    m2 = np.array([0, 1, 0, 1])
    c1 = np.stack([oracle.encrypt(p, rng, sk, int(m), 4, p.q) for m in m1])
    c2 = np.stack([oracle.encrypt(p, rng, sk, int(m), 4, p.q) for m in m2])
    for g, f in truth.items():
        out = o.eval_bin_gate(g, c1, c2)
        got = [oracle.decrypt(p, sk, r, 4, p.q) for r in out]
        assert got == [f(int(x), int(y)) for x, y in zip(m1, m2)], g


def test_keygen_stream_is_pinned(oracle):
    """or_keygen draws every key row from its own position of the one splitmix64 stream (counter-addressed, so
    the rows fill in parallel since round 6); the digests were recorded from the sequential round-5 walk, and
    the caller's stream continues after the keys exactly as it did."""
    op = oracle.params_from_set("TOY")
    r = oracle.Rng(31)
    sk, bsk, ksk = oracle.keygen(op, r)
    assert (oracle.fnv1a64(sk), oracle.fnv1a64(bsk), oracle.fnv1a64(ksk)) == (
        0x3045E07F7AFCD29, 0x7865F86830D66F63, 0x95776A0E9FA5F7EC)
    assert int(oracle.splitmix(r, 1, 1 << 62)[0]) == 1223636499923748511
