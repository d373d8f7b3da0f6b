"""GPU: the one-process multi-device path -- the reference's GPUSetup(numGPUs) (bootstrapping.cu:1005-1069)
with batches sharded over devices (bootstrapping.cu:1617, 1871) -- on the one-GPU development box.

TFHE_LOGICAL_DEVICES=k (an engine test hook, engine.hip create_ctx) presents k logical devices on the
one physical GPU, each with its own key arena, streams, scratch, pinned staging, completion flags and
host thread.  So the real multi-device code runs on real HIP: key replication (peer copies; RCCL is
used only between distinct devices), the contiguous shard split with ragged shards, one host thread
per device with concurrent launches, per-device flagged EvalAcc output, the row-pointer arrays, the
device-resident entry points' device choice, and chained bootstraps.  Every result must equal the
one-device context's bit for bit (which the oracle pins elsewhere).  The 1 -> 8 GPU run of bench.py is
the driver's (one process per GPU, RCCL broadcast of the key image).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pair(oracle):
    import os

    import tfhe_amd

    op = oracle.params_from_set("STD128")
    cp = tfhe_amd.params_from_set("STD128")
    rs = np.random.default_rng(2718)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    one = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk, num_gpus=1)
    os.environ["TFHE_LOGICAL_DEVICES"] = "3"
    try:
        multi = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk, num_gpus=3)
    finally:
        os.environ.pop("TFHE_LOGICAL_DEVICES", None)
    yield dict(op=op, one=one, multi=multi, rs=rs, tfhe=tfhe_amd)
    one.GPUClean()
    multi.GPUClean()


def test_three_logical_devices_replicated(pair):
    info = pair["multi"].info()
    assert info.num_devices == 3
    assert info.replicate_method == 2  # TFHE_REPLICATE_PEER (one GPU: no RCCL communicator)
    assert info.replicate_ms > 0


@pytest.mark.parametrize("B", [2, 7, 1001, 8192])
def test_sharded_gates_equal_one_device(pair, B):
    op, one, multi, rs = pair["op"], pair["one"], pair["multi"], pair["rs"]
    c1 = rs.integers(0, op.q, (B, op.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, op.q, (B, op.n + 1), dtype=np.uint64)
    for gate in ("NAND", "XOR"):
        assert np.array_equal(multi.EvalBinGate(gate, c1, c2), one.EvalBinGate(gate, c1, c2)), (gate, B)


def test_sharded_eval_acc_and_mkm_equal_one_device(pair):
    """EvalAcc takes the completion-flagged output path on every logical device at once (one flag
    array per device), the key switch the tiled form on the 2731-ciphertext shards."""
    op, one, multi, rs = pair["op"], pair["one"], pair["multi"], pair["rs"]
    B = 8193
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = np.zeros((B, 2, op.N), dtype=np.uint64)
    acc[:, 1, ::2] = rs.integers(0, op.Q, (B, op.N // 2), dtype=np.uint64)
    assert np.array_equal(multi.EvalAcc(a, op.q, acc), one.EvalAcc(a, op.q, acc))
    ext = rs.integers(0, op.Q, (B, op.N + 1), dtype=np.uint64)
    assert np.array_equal(multi.MKMSwitch(ext, op.q), one.MKMSwitch(ext, op.q))


def test_sharded_rows_api_equal_one_device(pair):
    from tfhe_amd.capi import check

    op, one, multi, rs, tf = pair["op"], pair["one"], pair["multi"], pair["rs"], pair["tfhe"]
    lib = tf.lib()
    B, tvlen = 3001, op.q // 2
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    tv = rs.integers(0, op.Q, (B, tvlen), dtype=np.uint64)
    want = np.empty((B, 2, op.N), dtype=np.uint64)
    check(lib.tfhe_eval_acc_tv(one.handle, B, a, op.q, tv, tvlen, want), "tfhe_eval_acc_tv")
    a_rows = [np.array(x) for x in a]
    rows = [np.empty(op.N, dtype=np.uint64) for _ in range(2 * B)]
    P = (C.c_void_p * len(a_rows))(*[x.ctypes.data for x in a_rows])
    R = (C.c_void_p * len(rows))(*[x.ctypes.data for x in rows])
    check(lib.tfhe_eval_acc_tv_rows(multi.handle, B, P, op.q, tv, tvlen, R), "tfhe_eval_acc_tv_rows")
    assert np.array_equal(np.stack(rows).reshape(B, 2, op.N), want)


def test_sharded_chained_sign_equal_one_device(pair):
    op, one, multi, rs = pair["op"], pair["one"], pair["multi"], pair["rs"]
    ct = rs.integers(0, 1 << 12, (301, op.n + 1), dtype=np.uint64)
    assert np.array_equal(multi.EvalSign(ct, 1 << 12), one.EvalSign(ct, 1 << 12))


def test_device_resident_call_on_multi_device_context(pair):
    """tfhe_*_device on a multi-device context: the call runs on the device holding the output buffer."""
    import torch

    op, one, multi, rs = pair["op"], pair["one"], pair["multi"], pair["rs"]
    B = 513
    c1 = rs.integers(0, op.q, (B, op.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, op.q, (B, op.n + 1), dtype=np.uint64)
    d1 = torch.from_numpy(c1.view(np.int64)).cuda()
    d2 = torch.from_numpy(c2.view(np.int64)).cuda()
    dout = torch.empty_like(d1)
    multi.EvalBinGateDevice("NAND", B, d1.data_ptr(), d2.data_ptr(), dout.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(dout.cpu().numpy().view(np.uint64), one.EvalBinGate("NAND", c1, c2))
