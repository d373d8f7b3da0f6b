"""GPU parity of the batch-tiled key switch (ks_tiled.hip) against the oracle's
ModSwitch -> KeySwitch -> ModSwitch (lwe-pke.cpp:204-215, 299-321).

Batches of >= ks_tiled_min (knob; TFHE_KS_TILED_MIN at setup) ciphertexts (default 256) take the tiled form, smaller
ones the per-ciphertext gather; both must equal the oracle bit for bit.  Every KSK word
width the engine packs is covered: u16 (STD128, qKS = 2^14), u32 with 32-bit sums
(STD192, qKS = 2^19, N dKS (qKS-1) < 2^32), u32 with 64-bit sums (STD128Q, qKS = 2^25)
and u64 (the logQ = 12 arbFunc context, qKS = 2^35, dKS = 7; since round 6 its tiled form runs on
split-word records, u32 + u8 per key, and the u64-word form stays as the ks40 = 0 cross-check).  Batches are ragged
(not multiples of the 512/1024-ciphertext tiles) and include all-zero and all-(Q-1)
extracts.  Random keys: bit-exactness does not need valid ones."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SETS = {
    "STD128": lambda m: m.params_from_set("STD128"),
    "STD192": lambda m: m.params_from_set("STD192"),
    "STD128Q": lambda m: m.params_from_set("STD128Q"),
    "ARB12": lambda m: m.params_from_logq("STD128", True, 12, 0, 0, 1),
    # round 4: the remaining tiled builds some parameter set reaches -- u16 keys with baseKS 32 (staging
    # depth 2), u32 keys with baseKS 64 (depth 8), u32 keys with u64 sums (qKS not a power of two)
    "STD128Q_OPT": lambda m: m.params_from_set("STD128Q_OPT"),
    "STD192Q": lambda m: m.params_from_set("STD192Q"),
    "SIGNED_MOD_TEST": lambda m: m.params_from_set("SIGNED_MOD_TEST"),
    # N = 8192 with u64 keys and dKS = 7: four waves' digit arrays exceed the LDS, so the gather runs
    # its one-wavefront form (k_mkm<uint64_t, 1>, lwe_kernels.hip)
    "TOY_N8192": lambda m: m.params_from_logq("TOY", False, 23, 8192, 0, 1),
}


@pytest.fixture(scope="module", params=list(SETS))
def ks_ctx(request, oracle):
    import tfhe_amd

    op = SETS[request.param](oracle)
    cp = SETS[request.param](tfhe_amd)
    rs = np.random.default_rng(31)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ksk.reshape(-1, cp.n + 1)[::97] = op.qKS - 1  # rows of maximal entries: the sums' upper bound
    ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    del bsk, ksk
    yield request.param, op, ctx, orc
    ctx.GPUClean()
    orc.close()


def _ext(op, B, seed):
    rs = np.random.default_rng(seed)
    ext = rs.integers(0, op.Q, (B, op.N + 1), dtype=np.uint64)
    ext[0, :] = 0
    ext[1, :] = op.Q - 1
    ext[B - 1, :] = op.Q // 2
    return ext


def _with_min(ctx, value, fn):
    """Run fn with the context's ks_tiled_min knob at value (TFHE_KS_TILED_MIN, read at setup)."""
    with ctx.knobs_set(ks_tiled_min=int(value)):
        return fn()


@pytest.mark.parametrize("B", [300, 1029])
def test_tiled_keyswitch_equals_oracle(ks_ctx, B):
    name, op, ctx, orc = ks_ctx
    ext = _ext(op, B, B)
    fmod = op.q
    tiled = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, fmod))
    gather = _with_min(ctx, "0", lambda: ctx.MKMSwitch(ext, fmod))
    assert np.array_equal(tiled, gather)
    # the oracle on a sample (all of them for the cheap STD128 key switch)
    idx = np.arange(B) if name == "STD128" else np.r_[0:6, B // 2 - 3:B // 2 + 3, B - 6:B]
    assert np.array_equal(tiled[idx], orc.mkm_switch(np.ascontiguousarray(ext[idx]), fmod))


def test_tiled_keyswitch_other_output_moduli(ks_ctx):
    name, op, ctx, orc = ks_ctx
    ext = _ext(op, 260, 7)
    idx = np.r_[0:4, 256:260]
    for fmod in (2 * op.q, 1 << 20, op.qKS):
        tiled = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, fmod))
        assert np.array_equal(tiled[idx], orc.mkm_switch(np.ascontiguousarray(ext[idx]), fmod)), fmod


def test_default_threshold_routes_small_batches_to_gather(ks_ctx):
    """Below the threshold (and for B = 1) the gather runs; results agree across the switch."""
    name, op, ctx, orc = ks_ctx
    ext = _ext(op, 255, 9)
    a = _with_min(ctx, "256", lambda: ctx.MKMSwitch(ext, op.q))
    b = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, op.q))
    assert np.array_equal(a, b)
    one = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext[:1], op.q))
    assert np.array_equal(one, orc.mkm_switch(np.ascontiguousarray(ext[:1]), op.q))


@pytest.mark.parametrize("cts", ["1", "2", "4"])
def test_tiled_keyswitch_ciphertexts_per_thread(ks_ctx, cts):
    """Every tile depth (one, two or -- the packed u16 form only, STD128's default from 2048 ciphertexts -- four
    ciphertexts per thread; the default picks by key width and batch) equals the gather form."""
    name, op, ctx, orc = ks_ctx
    if cts == "4" and not (op.qKS <= (1 << 16) and op.qKS & (op.qKS - 1) == 0):  # u16 keys, packed sums
        pytest.skip("four per thread: the packed u16 form only (other widths take two)")
    ext = _ext(op, 1029, 13)
    gather = _with_min(ctx, "0", lambda: ctx.MKMSwitch(ext, op.q))
    # 8-byte keys: both the split-word records (ks40 = 1, the default) and the u64 words at both depths
    for k40 in ((1, 0) if op.qKS > (1 << 32) else (1,)):
        with ctx.knobs_set(ks_cts=int(cts), ks40=k40):
            tiled = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, op.q))
        assert np.array_equal(tiled, gather), k40


def test_u16_keys_without_packed_sums(ks_ctx):
    """u16 keys with 32-bit column sums (the ks_pk knob 0) equal the packed-u16-sum form and the gather."""
    name, op, ctx, orc = ks_ctx
    if ctx.info().ksk_device_bytes == 0 or op.qKS > (1 << 16):
        pytest.skip("u16 keys only")
    ext = _ext(op, 700, 21)
    packed = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, op.q))
    with ctx.knobs_set(ks_pk=0):
        plain = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, op.q))
    gather = _with_min(ctx, "0", lambda: ctx.MKMSwitch(ext, op.q))
    assert np.array_equal(packed, plain) and np.array_equal(plain, gather)


@pytest.mark.parametrize("ks_ctx", ["ARB12"], indirect=True)
@pytest.mark.parametrize("B", [2, 128, 1029])
def test_split_word_keys_equal_u64_words(ks_ctx, B):
    """8-byte keys with qKS = 2^35 (ARB12 / the logQ contexts; TOY_N8192 takes the gather): the tiled key
    switch on the split-word records (ks40 = 1, the default: u32 low word + u8 high part, high parts summed
    as byte fields mod 2^3) equals the u64-word form, the gather and the oracle -- at B = 2 and 128 through
    the step split (partial sums + k_ks_combine), at 1029 without it; the rows of maximal entries (qKS - 1)
    put every byte field at its bound."""
    name, op, ctx, orc = ks_ctx
    assert op.qKS == (1 << 35) and ctx.knobs()["ks40"] == 1
    ext = _ext(op, B, 40 + B)
    split40 = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, op.q))
    with ctx.knobs_set(ks40=0):
        words = _with_min(ctx, "1", lambda: ctx.MKMSwitch(ext, op.q))
    gather = _with_min(ctx, "0", lambda: ctx.MKMSwitch(ext, op.q))
    assert np.array_equal(split40, words) and np.array_equal(words, gather)
    idx = np.unique(np.r_[0:min(B, 3), B - 1])
    assert np.array_equal(split40[idx], orc.mkm_switch(np.ascontiguousarray(ext[idx]), op.q))
