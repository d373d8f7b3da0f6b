#!/usr/bin/env python3
"""Blind rotation alone, device-resident, for same-box A/B of library builds (tools/alt_build.sh variants):

    python3 tools/br_ab.py --ctx LOGQ23 --batches 1024 [--lib altlib/X/libtfhe_hip_test.so] [--knob k=v ...]

One JSON line: per batch the min / mean of --reps timed launches (HIP stream sync) and a checksum of the output
accumulators after a fixed number of launches from a fixed input (equal checksums = equal outputs).
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-gpu_amd")]
CTX = {"STD128": ("set", "STD128"), "STD128Q": ("set", "STD128Q"), "STD192": ("set", "STD192"),
       "ARB12": ("logq", "STD128", True, 12, 0, 0, 1), "LOGQ23": ("logq", "STD128", False, 23, 0, 0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", default="LOGQ23", choices=list(CTX))
    ap.add_argument("--batches", default="1024")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--knob", action="append", default=[])
    args = ap.parse_args()
    import torch

    import tfhe_amd
    from bench import synthetic_keys

    spec = CTX[args.ctx]
    p = tfhe_amd.params_from_set(spec[1]) if spec[0] == "set" else tfhe_amd.params_from_logq(*spec[1:])
    bsk, ksk = synthetic_keys(p)
    ctx = tfhe_amd.BinFHEContextHIP(p, library=args.lib).GPUSetup(bsk, ksk)
    del bsk, ksk
    if args.knob:
        ctx.set_knobs(**{k: int(v) for k, v in (x.split("=") for x in args.knob)})
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    lib = ctx._L
    rows = []
    for B in (int(x) for x in args.batches.split(",")):
        g = torch.Generator(device=dev)
        g.manual_seed(B)
        a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
        acc = torch.randint(0, int(p.Q), (B, 2, p.N), dtype=torch.int64, device=dev, generator=g)
        ts = []
        for _ in range(args.reps + 1):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            tfhe_amd.capi.check(lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp),
                                "eval_acc")
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        ts = ts[1:]
        digest = hashlib.sha256(acc.cpu().numpy().tobytes()).hexdigest()[:16]
        rows.append({"B": B, "min_ms": round(min(ts) * 1e3, 3), "mean_ms": round(sum(ts) / len(ts) * 1e3, 3),
                     "digest": digest})
    print(json.dumps({"ctx": args.ctx, "lib": args.lib or "default", "knobs": args.knob, "rows": rows,
                      "duo_timeouts": int(ctx.info().duo_timeouts)}), flush=True)
    ctx.GPUClean()


if __name__ == "__main__":
    main()
