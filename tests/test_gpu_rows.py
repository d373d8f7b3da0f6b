"""GPU: the row-pointer host arrays (tfhe_eval_acc_tv_rows, tfhe_mkm_switch_rows) the drop-in shim
uses to hand OpenFHE's per-polynomial NativeVector storage to the PCIe staging in place.  They must
give exactly the flat calls' results -- which the oracle pins elsewhere -- for batches whose rows
straddle the 8 MiB pinned blocks, for ragged batch sizes, for both key-switch forms (gather below
4096 ciphertexts, tiled above), and when an unreduced input sends a row array again as u64."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi():
    import tfhe_amd

    return tfhe_amd


def check(st, where):
    from tfhe_amd.capi import check as _check

    _check(st, where)


def ptrs(arrs):
    return (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


@pytest.fixture(scope="module")
def std128(capi, oracle):
    op = oracle.params_from_set("STD128")
    cp = capi.params_from_set("STD128")
    rs = np.random.default_rng(77)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    yield dict(op=op, ctx=ctx, orc=orc, capi=capi)
    ctx.GPUClean()
    orc.close()


@pytest.mark.parametrize("B", [1, 37, 2600])
def test_eval_acc_tv_rows_equals_flat(std128, B):
    op, ctx, capi = std128["op"], std128["ctx"], std128["capi"]
    lib = capi.lib()
    rs = np.random.default_rng(B)
    amod = op.q
    tvlen = amod // 2
    a = rs.integers(0, amod, (B, op.n), dtype=np.uint64)
    tv = rs.integers(0, op.Q, (B, tvlen), dtype=np.uint64)
    flat = np.empty((B, 2, op.N), dtype=np.uint64)
    check(lib.tfhe_eval_acc_tv(ctx.handle, B, a, amod, tv, tvlen, flat), "tfhe_eval_acc_tv")
    # every row its own allocation, in shuffled order
    a_rows = [np.array(a[s]) for s in range(B)]
    acc_rows = [np.full(op.N, 0xDEADBEEF, dtype=np.uint64) for _ in range(2 * B)]
    check(lib.tfhe_eval_acc_tv_rows(ctx.handle, B, ptrs(a_rows), amod, tv, tvlen, ptrs(acc_rows)),
               "tfhe_eval_acc_tv_rows")
    got = np.stack(acc_rows).reshape(B, 2, op.N)
    assert np.array_equal(got, flat)
    if B <= 37:  # the flat call itself against the oracle on the expanded accumulators
        acc = np.zeros((B, 2, op.N), dtype=np.uint64)
        acc[:, 1, :: op.N // tvlen] = tv
        assert np.array_equal(flat, std128["orc"].eval_acc(a, amod, acc))


@pytest.mark.parametrize("B", [1, 37, 4500])
def test_mkm_switch_rows_equals_flat(std128, B):
    op, ctx, capi = std128["op"], std128["ctx"], std128["capi"]
    lib = capi.lib()
    rs = np.random.default_rng(1000 + B)
    ext = rs.integers(0, op.Q, (B, op.N + 1), dtype=np.uint64)
    want = ctx.MKMSwitch(ext, op.q)
    a_rows = [np.array(ext[s, : op.N]) for s in range(B)]
    b = np.array(ext[:, op.N])
    out_rows = [np.full(op.n, 7, dtype=np.uint64) for _ in range(B)]
    out_b = np.zeros(B, dtype=np.uint64)
    check(lib.tfhe_mkm_switch_rows(ctx.handle, B, ptrs(a_rows), b.ctypes.data, op.q, ptrs(out_rows),
                                        out_b.ctypes.data), "tfhe_mkm_switch_rows")
    got = np.concatenate([np.stack(out_rows), out_b[:, None]], axis=1)
    assert np.array_equal(got, want)
    if B <= 37:
        assert np.array_equal(want, std128["orc"].mkm_switch(ext, op.q))


def test_rows_unreduced_input_takes_the_wide_wire(std128):
    """A row value >= Q cannot cross in the u32 wire word: the runner resends the row array as u64,
    which must give the flat call's result on the same input."""
    op, ctx, capi = std128["op"], std128["ctx"], std128["capi"]
    lib = capi.lib()
    rs = np.random.default_rng(5)
    B = 9
    ext = rs.integers(0, op.Q, (B, op.N + 1), dtype=np.uint64)
    ext[4, 17] += np.uint64(op.Q) * np.uint64(1 << 20)
    want = ctx.MKMSwitch(ext, op.q)  # the flat call, whose wide-wire fallback test_gpu_parity covers
    a_rows = [np.array(ext[s, : op.N]) for s in range(B)]
    b = np.array(ext[:, op.N])
    out_rows = [np.zeros(op.n, dtype=np.uint64) for _ in range(B)]
    out_b = np.zeros(B, dtype=np.uint64)
    check(lib.tfhe_mkm_switch_rows(ctx.handle, B, ptrs(a_rows), b.ctypes.data, op.q, ptrs(out_rows),
                                        out_b.ctypes.data), "tfhe_mkm_switch_rows")
    got = np.concatenate([np.stack(out_rows), out_b[:, None]], axis=1)
    assert np.array_equal(got, want)


def test_rows_reject_null_rows(std128):
    ctx, capi = std128["ctx"], std128["capi"]
    op = std128["op"]
    lib = capi.lib()
    a_rows = (C.c_void_p * 2)(None, None)
    b = np.zeros(2, dtype=np.uint64)
    out = [np.zeros(op.n, dtype=np.uint64) for _ in range(2)]
    st = lib.tfhe_mkm_switch_rows(ctx.handle, 2, a_rows, b.ctypes.data, op.q, ptrs(out), b.ctypes.data)
    assert st == 1  # TFHE_ERR_INVALID_ARGUMENT


def test_flagged_eval_acc_output_equals_whole_launch_drain(std128, monkeypatch):
    """The host-array EvalAcc drains finished ciphertexts while its blind rotation still runs
    (completion flags, engine.hip d2h_flagged); the acc_flags knob 0 waits for the whole launch.  Both
    must return the same accumulators -- 8192 ciphertexts = 16 staging blocks, rows and flat."""
    op, ctx, capi = std128["op"], std128["ctx"], std128["capi"]
    lib = capi.lib()
    rs = np.random.default_rng(8192)
    B, amod = 8192, op.q
    tvlen = amod // 2
    a = rs.integers(0, amod, (B, op.n), dtype=np.uint64)
    tv = rs.integers(0, op.Q, (B, tvlen), dtype=np.uint64)
    outs = {}
    for flags in ("1", "0"):
        ctx.set_knobs(acc_flags=int(flags))
        flat = np.empty((B, 2, op.N), dtype=np.uint64)
        check(lib.tfhe_eval_acc_tv(ctx.handle, B, a, amod, tv, tvlen, flat), "tfhe_eval_acc_tv")
        acc_rows = [np.empty(op.N, dtype=np.uint64) for _ in range(2 * B)]
        check(lib.tfhe_eval_acc_tv_rows(ctx.handle, B, ptrs([x for x in a]), amod, tv, tvlen, ptrs(acc_rows)),
              "tfhe_eval_acc_tv_rows")
        assert np.array_equal(np.stack(acc_rows).reshape(B, 2, op.N), flat)
        outs[flags] = flat
    ctx.set_knobs(acc_flags=1)
    assert np.array_equal(outs["1"], outs["0"])
    # sampled against the oracle on the expanded accumulators
    idx = [0, 1, 511, 512, 4095, 8191]
    acc = np.zeros((len(idx), 2, op.N), dtype=np.uint64)
    acc[:, 1, :: op.N // tvlen] = tv[idx]
    assert np.array_equal(outs["1"][idx], std128["orc"].eval_acc(a[idx], amod, acc))
