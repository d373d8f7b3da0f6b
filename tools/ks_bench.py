#!/usr/bin/env python3
"""Key-switch (MKM) kernel A/B on one MI355X: the per-ciphertext gather (k_mkm) against
the batch-tiled form (ks_tiled.hip), device-resident inputs, HIP events on the launch
stream.  Both outputs must be equal.  One JSON line per configuration.
Usage: python3 tools/ks_bench.py [STD128 STD192 STD128Q ARB12 LOGQ23] [--reps 3] [--batches 1,16,128]
                                 [--splits 4,16]
--batches sweeps the batch (one context per configuration); --splits times the tiled form at each
ks_split cap (the knob; the engine caps it at 4 above 512 ciphertexts).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))

CONFIGS = {  # name: (params, batch of the BASELINE configuration that uses it)
    "STD128": (lambda c: c.params_from_set("STD128"), 8192),
    "STD192": (lambda c: c.params_from_set("STD192"), 8192),
    "STD128Q": (lambda c: c.params_from_set("STD128Q"), 1024),
    "ARB12": (lambda c: c.params_from_logq("STD128", True, 12, 0, 0, 1), 4096),
    "LOGQ23": (lambda c: c.params_from_logq("STD128", False, 23, 0, 0, 1), 1024),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=list(CONFIGS))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="override the batch")
    ap.add_argument("--batches", default="", help="comma-separated batch sweep")
    ap.add_argument("--splits", default="32", help="comma-separated ks_split caps for the tiled form")
    ap.add_argument("--ks40", default="0,1", help="ks40 knob values timed for the tiled form (8-byte keys: the u64 "
                                                 "words = 0, the split-word records = 1; ignored elsewhere)")
    args = ap.parse_args()
    import torch

    import tfhe_amd
    from tfhe_amd import capi

    for name in args.configs:
        mk, B0 = CONFIGS[name]
        batches = [int(x) for x in args.batches.split(",")] if args.batches else [args.batch or B0]
        p = mk(capi)
        rs = np.random.default_rng(3)
        bsk = rs.integers(0, p.Q, p.bsk_words(), dtype=np.uint64)
        ksk = rs.integers(0, p.qKS, p.ksk_words(), dtype=np.uint64)
        ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
        del bsk, ksk
        full = torch.from_numpy(rs.integers(0, p.Q, (max(batches), p.N + 1), dtype=np.uint64).view(np.int64)).cuda()
        s = torch.cuda.Stream()
        for B in batches:
            ext = full[:B].contiguous()
            outs = {}
            res = {"config": name, "batch": B, "N": p.N, "n": p.n, "qKS": p.qKS, "baseKS": p.baseKS, "dKS": p.dKS}
            k40 = [int(x) for x in args.ks40.split(",")] if p.qKS > (1 << 32) else [1]
            modes = [("gather", 0, 16, 1)] + [(f"tiled_split{z}" + (f"_ks40{k}" if len(k40) > 1 else ""), 1, int(z), k)
                                              for z in args.splits.split(",") for k in k40]
            for mode, tmin, split, k in modes:
                ctx.set_knobs(ks_tiled_min=tmin, ks_split=split, ks40=k)
                out = torch.empty((B, p.n + 1), dtype=torch.int64, device="cuda")
                call = lambda: capi.check(capi.lib().tfhe_mkm_switch_device(ctx.handle, B, ext.data_ptr(), p.q,
                                                                            out.data_ptr(), s.cuda_stream), "mkm")
                call()
                s.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(args.reps):
                    call()
                e1.record(s)
                s.synchronize()
                outs[mode] = out.cpu().numpy()
                res[f"{mode}_ms"] = round(e0.elapsed_time(e1) / args.reps, 3)
            ctx.set_knobs(ks_tiled_min=-1, ks_split=32, ks40=1)
            res["equal"] = all(np.array_equal(outs["gather"], v) for v in outs.values())
            print(json.dumps(res), flush=True)
        ctx.GPUClean()
        del full

if __name__ == "__main__":
    main()
