"""GPU: the one-digit special-form blind rotation on two workgroups per ciphertext (k_blind_rotate_sfduo<1>,
blind_rotate_generic.hip; verdict r5 "missing" 2).

C3's context class (arbFunc logQ 12: Q = 2^54 - 77823, N = 2048, one transformed digit after one thrown)
runs batches of at most tfhe_knobs.duo (default 128) ciphertexts -- and at most the device's co-resident
pairs -- with each ciphertext's round split by NTT half over two workgroups that exchange 16 KiB per round
through memory.  Checked through the C-ABI:
  * EvalAcc bit-exact against the oracle at batches that leave pair groups ragged (1, 7, 9) and at boundary
    accumulator coefficients and rotations;
  * the same outputs as the one-workgroup sf2<1> (duo = 0) at 64 and 128, and 129 (past the co-resident
    pairs: one workgroup per ciphertext);
  * EvalFunc (m^3 mod 8, the bench's C3 function) at 128 with valid keys: duo = one workgroup = oracle on a
    sample, and every output decrypts;
  * a partner that never arrives (test library, probe 5): both members time out, the rescue launch recomputes
    the ciphertext, every output stays exact;
  * no partner times out otherwise (tfhe_info.duo_timeouts).
Keys: the Appendix B splitmix64 keys (parity does not need valid keys; the session's shared contexts); the
EvalFunc case uses the oracle's keygen.
"""
import numpy as np
import pytest

from helpers import cube_lut

pytestmark = pytest.mark.gpu
SPEC = ("STD128", True, 12, 0, 0, 1)


@pytest.fixture(scope="module")
def sfd(shared_kat):
    s = shared_kat("ARB12")
    cp, ctx = s["cp"], s["ctx"]
    assert cp.digitsG - cp.numDigitsToThrow == 1 and cp.N == 2048 and cp.Q == (1 << 54) - 77823
    assert ctx.info().br_kernel == 5 and ctx.knobs()["duo"] == 128  # TFHE_BR_SF
    yield s
    assert ctx.info().duo_timeouts == 0


def _inputs(op, B, seed):
    rs = np.random.default_rng(seed)
    return (rs.integers(0, 2 * op.N, (B, op.n), dtype=np.uint64),
            rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64))


@pytest.mark.parametrize("B", [1, 7, 9])
def test_sfduo_eval_acc_matches_oracle(sfd, B):
    op, ctx, orc = sfd["op"], sfd["ctx"], sfd["orc"]
    a, acc = _inputs(op, B, 500 + B)
    out = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(out.reshape(B, -1), orc.eval_acc(a, 2 * op.N, acc).reshape(B, -1))
    assert ctx.info().duo_timeouts == 0


def test_sfduo_boundary_coefficients(sfd):
    """Accumulators at the decomposition's edges (0, 1, Q/2 - 1, Q/2, Q/2 + 1, Q - 1; the digit's sign flips at
    Q/2) and rotations 0, N and the extremes of [0, 2N)."""
    op, ctx, orc = sfd["op"], sfd["ctx"], sfd["orc"]
    Q, h = op.Q, op.Q // 2
    edge = np.array([0, 1, h - 1, h, h + 1, Q - 1], dtype=np.uint64)
    rs = np.random.default_rng(601)
    B = 3
    acc = edge[rs.integers(0, len(edge), (B, 2, op.N))]
    a = rs.integers(0, 2 * op.N, (B, op.n), dtype=np.uint64)
    a[0, :] = 0
    a[1, ::2] = op.N
    a[2, ::3] = 2 * op.N - 1
    out = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(out.reshape(B, -1), orc.eval_acc(a, 2 * op.N, acc).reshape(B, -1))


@pytest.mark.parametrize("B", [64, 128, 129])
def test_sfduo_equals_one_workgroup_form(sfd, B):
    """duo = 256 (the knob's maximum): 64 and 128 run sfduo<1>; 129 is past the device's co-resident pairs (one
    132-KiB workgroup per CU: half of MI355X's 256 CUs) and runs sf2<1>; every form equals duo = 0 and the
    oracle on three ciphertexts."""
    op, ctx = sfd["op"], sfd["ctx"]
    a, acc = _inputs(op, B, 700 + B)
    with ctx.knobs_set(duo=256):
        two = ctx.EvalAcc(a, 2 * op.N, acc)
    with ctx.knobs_set(duo=0):
        one = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(two, one)
    idx = [0, B // 2, B - 1]
    assert np.array_equal(two[idx].reshape(3, -1), sfd["orc"].eval_acc(a[idx], 2 * op.N, acc[idx]).reshape(3, -1))


def test_sfduo_evalfunc_decrypts(oracle):
    """EvalFunc(m^3 mod 8) on 128 ciphertexts (C3's function at the duo batch): the duo form equals the
    one-workgroup form and the oracle on a sample, and every output decrypts to f(m)."""
    import tfhe_amd

    op, cp = oracle.params_from_logq(*SPEC), tfhe_amd.params_from_logq(*SPEC)
    rng = oracle.Rng(35)
    sk, bsk, ksk = oracle.keygen(op, rng)
    ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    del bsk, ksk
    try:
        P = 8
        lut = cube_lut(cp.q, P)
        ms = np.random.default_rng(3).integers(0, P, 128)
        ct = np.stack([oracle.encrypt(op, rng, sk, int(m), P, op.q) for m in ms])
        out = ctx.EvalFunc(ct, lut)
        with ctx.knobs_set(duo=0):
            ref = ctx.EvalFunc(ct, lut)
        assert np.array_equal(out, ref)
        assert np.array_equal(out[[0, 101]], orc.eval_func(ct[[0, 101]], lut))
        assert [oracle.decrypt(op, sk, r, P, op.q) for r in out] == [int(m) ** 3 % P for m in ms]
        assert ctx.info().duo_timeouts == 0
    finally:
        ctx.GPUClean()
        orc.close()


def test_sfduo_partner_timeout_is_recomputed(shared_kat):
    """The test library's probe 5 makes member 1 of pair 0 stop publishing at round 2: both members time out,
    the pair's failed word is set, and the rescue (k_blind_rotate_sf2<1, true>) recomputes that ciphertext from
    its saved input -- every output stays bit-exact and tfhe_info.duo_timeouts counts the two workgroups."""
    s = shared_kat("ARB12", test_lib=True)
    op, ctx, orc = s["op"], s["ctx"], s["orc"]
    a, acc = _inputs(op, 9, 800)
    want = orc.eval_acc(a, 2 * op.N, acc)
    t0 = ctx.info().duo_timeouts
    assert np.array_equal(ctx.EvalAcc(a, 2 * op.N, acc), want)
    assert ctx.info().duo_timeouts == t0
    with ctx.knobs_set(probe=5):
        got = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(got, want)
    assert ctx.info().duo_timeouts == t0 + 2
    assert np.array_equal(ctx.EvalAcc(a, 2 * op.N, acc), want)
    assert ctx.info().duo_timeouts == t0 + 2
