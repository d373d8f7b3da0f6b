#!/usr/bin/env python3
"""Host-array entry point (the drop-in boundary: host buffers in and out, PCIe inside the
timed call) against the device-resident entry point on the same box, STD128 NAND.
Usage: python3 tools/host_path_bench.py [--batch 8192] [--reps 5]
The host_parts knob (sub-batches per device) is set per variant through tfhe_set_knobs."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--parts", default="1,2,4")
    args = ap.parse_args()
    import torch

    import tfhe_amd
    from tfhe_amd import capi

    p = capi.params_from_set("STD128")
    rs = np.random.default_rng(1)
    bsk = rs.integers(0, p.Q, p.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, p.qKS, p.ksk_words(), dtype=np.uint64)
    ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
    B = args.batch
    c1 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    d1 = torch.from_numpy(c1.view(np.int64)).cuda()
    d2 = torch.from_numpy(c2.view(np.int64)).cuda()
    do = torch.empty_like(d1)
    s = torch.cuda.Stream()
    res = {"batch": B}

    def dev():
        ctx.EvalBinGateDevice("NAND", B, d1.data_ptr(), d2.data_ptr(), do.data_ptr(), stream=s.cuda_stream)
        s.synchronize()

    out = np.empty((B, p.n + 1), dtype=np.uint64)

    def host():
        capi.check(capi.lib().tfhe_eval_bin_gate(ctx.handle, 3, B, c1.ravel(), c2.ravel(), p.q, out.ravel()), "gate")

    def timeit(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        return (time.perf_counter() - t0) / args.reps

    for rnd in range(2):  # alternate, so box drift hits every variant
        res.setdefault("device_ms", []).append(round(timeit(dev) * 1e3, 2))
        for parts in args.parts.split(","):
            ctx.set_knobs(host_parts=int(parts))
            res.setdefault(f"host_parts{parts}_ms", []).append(round(timeit(host) * 1e3, 2))
    ref = ctx.EvalBinGate("NAND", c1[:64], c2[:64])
    res["host_equals_device"] = bool(np.array_equal(out[:64], ref)) and bool(
        np.array_equal(do.cpu().numpy().view(np.uint64)[:64], ref))
    for k in list(res):
        if k.endswith("_ms"):
            res[k.replace("_ms", "_bootstraps_per_s")] = round(B / (min(res[k]) / 1e3), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
