"""GPU: the two-workgroup two-digit special-form blind rotation (k_blind_rotate_sfduo<2>, blind_rotate_generic.hip;
round 6: split by NTT half -- the round-4/5 form split by accumulator polynomial, k_blind_rotate_sf2duo, is the test
library's A/B form and is checked against it below).

Two-digit special-form contexts (C5b: STD128 logQ = 23, throw = 1) run batches of at most
`tfhe_knobs.duo` (default 128, at most 256) ciphertexts with each ciphertext's round split over two workgroups
that exchange 16 KiB per round through memory.  Checked here, through the C-ABI:
  * EvalAcc bit-exact against the oracle at batches that leave pair groups ragged (1, 7, 9) --
    the grid pairs blocks b and b + 8, so these exercise the exit of unused pairs;
  * the same outputs as the one-workgroup sf2 (duo = 0) at 64, 255 and 256 ciphertexts, and the
    first 256 ciphertexts of a 257-batch (which runs one workgroup per ciphertext);
  * EvalSign (7 chained bootstraps per sign) at the 8-GPU node's per-GPU shard of C5, 128;
  * no partner ever timed out (tfhe_info.duo_timeouts).
Keys are the Appendix B splitmix64 keys (parity does not need valid keys); the decrypting EvalSign
case uses the oracle's keygen.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
QIN = 1 << 23


def _ctx_params(mod):
    return mod.params_from_logq("STD128", False, 23, 0, 0, 1)


@pytest.fixture(scope="module")
def duo(shared_kat):
    s = shared_kat("LOGQ23")
    cp, ctx = s["cp"], s["ctx"]
    assert (cp.digitsG - cp.numDigitsToThrow) == 2 and cp.N == 2048  # the sf2<2> / sfduo<2> shape
    assert ctx.knobs()["duo"] == 128
    yield s
    assert ctx.info().duo_timeouts == 0


def _inputs(op, B, seed):
    rs = np.random.default_rng(seed)
    a = rs.integers(0, 2 * op.N, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    return a, acc


@pytest.mark.parametrize("B", [1, 7, 9])
def test_duo_eval_acc_matches_oracle(duo, B):
    op, ctx, orc = duo["op"], duo["ctx"], duo["orc"]
    a, acc = _inputs(op, B, 100 + B)
    out = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(out.reshape(B, -1), orc.eval_acc(a, 2 * op.N, acc).reshape(B, -1))
    assert ctx.info().duo_timeouts == 0


@pytest.mark.parametrize("B", [64, 128, 129])
def test_duo_equals_one_workgroup_form(duo, B):
    """duo = 256 (the knob's maximum): 64 and 128 run sfduo<2>; 129 is past the device's co-resident pairs (one
    148-KiB duo workgroup per CU: half of MI355X's 256 CUs), so it runs the one-workgroup kernel (a
    pair must never wait behind its own launch's pairs); every form equals duo = 0 and the oracle."""
    op, ctx = duo["op"], duo["ctx"]
    a, acc = _inputs(op, B, 200 + B)
    with ctx.knobs_set(duo=256):
        two = ctx.EvalAcc(a, 2 * op.N, acc)
    with ctx.knobs_set(duo=0):
        one = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(two, one)
    idx = [0, B // 2, B - 1]
    assert np.array_equal(two[idx].reshape(3, -1), duo["orc"].eval_acc(a[idx], 2 * op.N, acc[idx]).reshape(3, -1))


def test_duo_batch_limit(duo):
    """257 ciphertexts run one workgroup each; their first 256 equal the 256-batch run (which the co-residency cap
    also keeps on one workgroup per ciphertext); the knob itself stops at the exchange buffers' 256 pairs."""
    op, ctx = duo["op"], duo["ctx"]
    a, acc = _inputs(op, 257, 300)
    with ctx.knobs_set(duo=256):
        full = ctx.EvalAcc(a, 2 * op.N, acc)
        part = ctx.EvalAcc(a[:256], 2 * op.N, acc[:256])
    assert np.array_equal(full[:256], part)
    with pytest.raises(Exception):
        ctx.set_knobs(duo=257)  # the exchange buffers hold 256 pairs


def test_duo_evalsign_shard_decrypts(oracle):
    """EvalSign at C5's per-GPU shard of an 8-GPU node (1024 / 8 = 128): duo = one-workgroup form =
    oracle on a sample, and every output decrypts to the sign away from the boundaries."""
    import tfhe_amd

    op, cp = _ctx_params(oracle), _ctx_params(tfhe_amd)
    rng = oracle.Rng(32)
    sk, bsk, ksk = oracle.keygen(op, rng)
    ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    del bsk, ksk
    try:
        p = (op.q // 128 // 2) * (QIN // op.q)
        rs = np.random.default_rng(9)
        ms = rs.integers(0, p, 128)
        ct = np.stack([oracle.encrypt(op, rng, sk, int(m), p, QIN) for m in ms])
        out = ctx.EvalSign(ct, QIN)
        with ctx.knobs_set(duo=0):
            ref = ctx.EvalSign(ct, QIN)
        assert np.array_equal(out, ref)
        assert np.array_equal(out[[0, 77]], orc.eval_sign(ct[[0, 77]], QIN))
        dec = np.array([oracle.decrypt(op, sk, r, 2, op.q) for r in out])
        dist = np.minimum(np.abs(ms - p // 2), np.minimum(ms, p - ms))
        bad = np.flatnonzero(dec != (ms >= p // 2))
        assert np.all(dist[bad] < 8), (bad, ms[bad])
        assert ctx.info().duo_timeouts == 0
    finally:
        ctx.GPUClean()
        orc.close()


def test_duo_partner_timeout_is_recomputed(shared_kat):
    """A partner that never arrives: the test library's probe 5 makes member 1 of pair 0 stop
    publishing at round 2.  Both members time out, the pair's failed word is set, and the rescue launch
    behind the duo kernel recomputes that ciphertext from its saved input with the one-workgroup kernel:
    every output stays bit-exact and tfhe_info.duo_timeouts counts the two timed-out workgroups."""
    s = shared_kat("LOGQ23", test_lib=True)
    op, ctx, orc = s["op"], s["ctx"], s["orc"]
    a, acc = _inputs(op, 9, 400)
    want = orc.eval_acc(a, 2 * op.N, acc)
    t0 = ctx.info().duo_timeouts
    assert np.array_equal(ctx.EvalAcc(a, 2 * op.N, acc), want)
    assert ctx.info().duo_timeouts == t0
    with ctx.knobs_set(probe=5):
        got = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(got, want)
    assert ctx.info().duo_timeouts == t0 + 2
    assert np.array_equal(ctx.EvalAcc(a, 2 * op.N, acc), want)  # the failed word is cleared per launch
    assert ctx.info().duo_timeouts == t0 + 2


def test_polynomial_split_form_equals_default(shared_kat):
    """The test library's probe 13 runs the round-4/5 two-digit duo (k_blind_rotate_sf2duo, split by accumulator
    polynomial; 1.5-2.4 % slower than sfduo<2> at 128, profiles/r06m): the same outputs as the default form, the
    one-workgroup form and the oracle."""
    s = shared_kat("LOGQ23", test_lib=True)
    op, ctx, orc = s["op"], s["ctx"], s["orc"]
    a, acc = _inputs(op, 128, 450)
    t0 = ctx.info().duo_timeouts
    dflt = ctx.EvalAcc(a, 2 * op.N, acc)
    with ctx.knobs_set(probe=13):
        poly = ctx.EvalAcc(a, 2 * op.N, acc)
    with ctx.knobs_set(duo=0):
        one = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(dflt, poly) and np.array_equal(dflt, one)
    assert np.array_equal(dflt[[5]].reshape(1, -1), orc.eval_acc(a[[5]], 2 * op.N, acc[[5]]).reshape(1, -1))
    assert ctx.info().duo_timeouts == t0
