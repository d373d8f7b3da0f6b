#!/usr/bin/env python3
"""Timing probe: can the key switch of one half batch hide under the blind rotation of the other?
Two contexts on one GPU (separate arenas and scratch, so their calls may run concurrently), STD128,
B = 8192 accumulators.  Serial: EvalAcc(8192) then MKMSwitch(8192) on one stream.  Split: EvalAcc(H1)
+ MKMSwitch(H1) on a high-priority stream, EvalAcc(H2) + MKMSwitch(H2) on a low-priority stream,
both queued at once.  Outputs of both forms must be equal.  Prints one JSON line.
Usage: python3 tools/overlap_probe.py [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8192)
    args = ap.parse_args()
    import torch

    import tfhe_amd
    from tfhe_amd import capi

    p = tfhe_amd.params_from_set("STD128")
    rs = np.random.default_rng(5)
    bsk = rs.integers(0, p.Q, p.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, p.qKS, p.ksk_words(), dtype=np.uint64)
    ca = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
    cb = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
    B, H = args.batch, args.batch // 2
    a = torch.from_numpy(rs.integers(0, p.q, (B, p.n), dtype=np.uint64).view(np.int64)).cuda()
    acc0 = torch.from_numpy(rs.integers(0, p.Q, (B, 2, p.N), dtype=np.uint64).view(np.int64)).cuda()
    acc = torch.empty_like(acc0)
    ext = torch.empty((B, p.N + 1), dtype=torch.int64, device="cuda")
    out = torch.empty((B, p.n + 1), dtype=torch.int64, device="cuda")
    L = capi.lib()
    s0 = torch.cuda.Stream()
    hi, lo = torch.cuda.Stream(priority=-1), torch.cuda.Stream(priority=0)

    def ptr(t, row):
        return t.data_ptr() + row * t.stride(0) * 8

    def extract(lo_, cnt, s):  # (acc0 transposed, acc1[0]) as ext rows: a torch copy on stream s
        with torch.cuda.stream(s):
            ext[lo_:lo_ + cnt, :p.N] = acc[lo_:lo_ + cnt, 0, :]
            ext[lo_:lo_ + cnt, p.N] = acc[lo_:lo_ + cnt, 1, 0]

    def serial():
        acc.copy_(acc0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        capi.check(L.tfhe_eval_acc_device(ca.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), s0.cuda_stream), "acc")
        extract(0, B, s0)
        capi.check(L.tfhe_mkm_switch_device(ca.handle, B, ext.data_ptr(), int(p.q), out.data_ptr(), s0.cuda_stream), "mkm")
        e1.record(s0)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    def split():
        acc.copy_(acc0)
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(s0)
        hi.wait_event(e0)
        lo.wait_event(e0)
        for ctx, s, lo_ in ((ca, hi, 0), (cb, lo, H)):
            capi.check(L.tfhe_eval_acc_device(ctx.handle, H, ptr(a, lo_), int(p.q), ptr(acc, lo_), s.cuda_stream), "acc")
        for ctx, s, lo_ in ((ca, hi, 0), (cb, lo, H)):
            extract(lo_, H, s)
            capi.check(L.tfhe_mkm_switch_device(ctx.handle, H, ptr(ext, lo_), int(p.q), ptr(out, lo_), s.cuda_stream),
                       "mkm")
        e1.record(hi)
        e2.record(lo)
        torch.cuda.synchronize()
        return max(e0.elapsed_time(e1), e0.elapsed_time(e2))

    serial()
    ref = out.clone()
    split()
    equal = bool(torch.equal(out, ref))
    ts, tp = [], []
    for _ in range(args.reps):  # alternate
        ts.append(serial())
        tp.append(split())
    print(json.dumps({"batch": B, "serial_ms": [round(x, 3) for x in ts], "split_ms": [round(x, 3) for x in tp],
                      "serial_best": round(min(ts), 3), "split_best": round(min(tp), 3), "equal": equal}), flush=True)
    ca.GPUClean()
    cb.GPUClean()


if __name__ == "__main__":
    main()
