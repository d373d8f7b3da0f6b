"""GPU: the in-process RCCL replication branch of tfhe_setup(num_gpus) (engine.hip replicate_arena; the
reference replicates keys host-to-device per GPU, bootstrapping.cu:1005-1069), run on the one-GPU box.

A real communicator cannot hold one GPU twice, so with TFHE_LOGICAL_DEVICES the engine normally takes
the peer-copy path.  TFHE_RCCL_LIB selects a stub of the six RCCL entry points
(tests/stub_rccl/stub_rccl.cpp: broadcasts as HIP device copies ordered after the root's stream,
issued at ncclGroupEnd) so the engine's communicator / group / broadcast / sync / destroy sequence runs
for real; the result must equal a one-device context bit for bit.  Also: a failing ncclCommInitAll
falls back to peer copies, and a short broadcast is caught by the replica checksum at setup.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
STUB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stub_rccl", "librccl_stub.so")


def _setup(tfhe_amd, cp, bsk, ksk, devices, fail=None):
    env = {"TFHE_LOGICAL_DEVICES": str(devices), "TFHE_RCCL_LIB": STUB}
    if fail:
        env["STUB_RCCL_FAIL"] = fail
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk, num_gpus=devices)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def keys(oracle):
    import tfhe_amd

    cp = tfhe_amd.params_from_set("STD128")
    rs = np.random.default_rng(4242)
    bsk = rs.integers(0, cp.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, cp.qKS, cp.ksk_words(), dtype=np.uint64)
    one = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk, num_gpus=1)
    yield tfhe_amd, cp, bsk, ksk, one, rs
    one.GPUClean()


@pytest.mark.skipif(not os.path.exists(STUB), reason="tests/stub_rccl/librccl_stub.so not built")
def test_rccl_branch_replicates_and_matches_one_device(keys):
    tfhe_amd, cp, bsk, ksk, one, rs = keys
    stub = C.CDLL(STUB)  # the library the engine dlopen'ed (same handle: shared counters)
    b0, g0 = stub.stub_rccl_broadcasts(), stub.stub_rccl_groups()
    multi = _setup(tfhe_amd, cp, bsk, ksk, 3)
    try:
        info = multi.info()
        assert info.num_devices == 3
        assert info.replicate_method == 1  # TFHE_REPLICATE_RCCL
        assert stub.stub_rccl_broadcasts() - b0 == 2 and stub.stub_rccl_groups() - g0 == 1
        B = 1001
        c1 = rs.integers(0, cp.q, (B, cp.n + 1), dtype=np.uint64)
        c2 = rs.integers(0, cp.q, (B, cp.n + 1), dtype=np.uint64)
        assert np.array_equal(multi.EvalBinGate("NAND", c1, c2), one.EvalBinGate("NAND", c1, c2))
        lut = np.array([(3 * x) % cp.q for x in range(cp.q)], dtype=np.uint64)  # LUT per device, by index
        assert np.array_equal(multi.EvalFunc(c1, lut), one.EvalFunc(c1, lut))
    finally:
        multi.GPUClean()


@pytest.mark.skipif(not os.path.exists(STUB), reason="tests/stub_rccl/librccl_stub.so not built")
def test_failed_communicator_falls_back_to_peer_copies(keys):
    tfhe_amd, cp, bsk, ksk, one, rs = keys
    multi = _setup(tfhe_amd, cp, bsk, ksk, 2, fail="init")
    try:
        assert multi.info().replicate_method == 2  # TFHE_REPLICATE_PEER
        c1 = rs.integers(0, cp.q, (64, cp.n + 1), dtype=np.uint64)
        c2 = rs.integers(0, cp.q, (64, cp.n + 1), dtype=np.uint64)
        assert np.array_equal(multi.EvalBinGate("AND", c1, c2), one.EvalBinGate("AND", c1, c2))
    finally:
        multi.GPUClean()


@pytest.mark.skipif(not os.path.exists(STUB), reason="tests/stub_rccl/librccl_stub.so not built")
def test_short_broadcast_fails_setup(keys):
    tfhe_amd, cp, bsk, ksk, one, rs = keys
    with pytest.raises(tfhe_amd.TfheError, match="replica on device 1 differs"):
        _setup(tfhe_amd, cp, bsk, ksk, 2, fail="short")
