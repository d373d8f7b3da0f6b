"""GPU: the device-resident fused EvalFunc / EvalFloor entry points (tfhe_eval_func_device,
tfhe_eval_floor_device; ABI 5) -- the pipelines of the host-array calls with inputs, LUTs and outputs in
HBM, ordered on a caller stream.  Each equals the host-array call and the oracle bit for bit, for the
three LUT classes of checkInputFunction (binfhe-base-scheme.cpp:162-186: negacyclic, periodic,
arbitrary) and per-ciphertext LUTs, on the C3 context (logQ = 12 arbFunc, throw = 1: sf2) and STD128
(fast4)."""
import numpy as np
import pytest

from helpers import cube_lut

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["STD128", "arb12"])
def env(request, shared_kat):
    s = shared_kat("STD128" if request.param == "STD128" else "ARB12")  # the session's shared contexts
    return s["op"], s["ctx"], s["orc"]


def _dev(x):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x).astype(np.int64)).to(torch.device("cuda", 0))


def _luts(q):
    h = q // 2  # lut[i] == q - lut[h + i] for every i < h (checkInputFunction's negacyclic test)
    neg = np.array([1 + (3 * x) % (q - 1) if x < h else q - 1 - (3 * (x - h)) % (q - 1) for x in range(q)],
                   dtype=np.uint64)
    per = np.array([(x * 5) % (q // 2) for x in range(q)], dtype=np.uint64)
    return {"negacyclic": neg, "periodic": per, "arbitrary": cube_lut(q)}


@pytest.mark.parametrize("kind", ["negacyclic", "periodic", "arbitrary", "per_ct"])
def test_eval_func_device(env, kind):
    import torch

    op, ctx, orc = env
    q = op.q
    if kind == "arbitrary" and q > op.N:
        pytest.skip("arbitrary LUTs need q <= N")
    rs = np.random.default_rng(11)
    B = 67
    ct = rs.integers(0, q, (B, op.n + 1), dtype=np.uint64)
    if kind == "per_ct":
        lut = np.stack([_luts(q)["periodic"]] + [rs.integers(0, q, q, dtype=np.uint64) for _ in range(B - 1)])
    else:
        lut = _luts(q)[kind]
    s = torch.cuda.Stream(torch.device("cuda", 0))
    d, dl = _dev(ct), _dev(lut)
    do = torch.empty_like(d)
    ctx.EvalFuncDevice(B, d.data_ptr(), dl.data_ptr(), do.data_ptr(), per_ct_lut=lut.ndim == 2, stream=s.cuda_stream)
    torch.cuda.synchronize()
    got = do.cpu().numpy().astype(np.uint64)
    assert np.array_equal(got, ctx.EvalFunc(ct, lut))
    idx = [0, B - 1]
    want = orc.eval_func(ct[idx], lut[idx] if lut.ndim == 2 else lut)
    assert np.array_equal(got[idx], want)


def test_eval_floor_device(env):
    import torch

    op, ctx, orc = env
    rs = np.random.default_rng(12)
    B = 33
    ct = rs.integers(0, op.q, (B, op.n + 1), dtype=np.uint64)
    d = _dev(ct)
    do = torch.empty_like(d)
    ctx.EvalFloorDevice(B, d.data_ptr(), op.q, do.data_ptr(), roundbits=1)
    torch.cuda.synchronize()
    got = do.cpu().numpy().astype(np.uint64)
    assert np.array_equal(got, ctx.EvalFloor(ct, op.q, 1))
    assert np.array_equal(got[:2], orc.eval_floor(ct[:2], op.q, 1))
