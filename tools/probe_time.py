#!/usr/bin/env python3
"""Upper bounds of two round-6 levers, timed on the test library (lib/libtfhe_hip_test.so) as the
device-resident blind rotation (min of --reps, stream-synchronised), one JSON line:
  f64wduo  STD128Q at 128 ciphertexts (C5a's 8-GPU shard): default against probe 11 = no D / C' exchange
           barrier (results invalid) -- what removing that barrier by a new thread mapping could gain at most
  sf2p     logQ = 23 at 1024 (C5b): default against probe 12 = wave-uniform factor-table rows (results
           invalid) -- what the table's LDS bank conflicts cost at most
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-gpu_amd")]


def timed(ctx, lib, p, B, knobs, reps, dev, sp, g):
    import torch

    import tfhe_amd

    a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
    acc0 = torch.randint(0, int(p.Q), (B, 2, p.N), dtype=torch.int64, device=dev, generator=g)
    acc = acc0.clone()
    ts = []
    with ctx.knobs_set(**knobs):
        for _ in range(reps + 1):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            tfhe_amd.capi.check(lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp),
                                "eval_acc")
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
    return round(min(ts[1:]) * 1e3, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--which", default="f64wduo,sf2p")
    args = ap.parse_args()
    import torch

    import tfhe_amd
    from bench import synthetic_keys

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    lib = tfhe_amd.lib(tfhe_amd.capi.TEST_LIB)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    out = {"what": "round-6 lever bounds (timing-only probes, results invalid)", "rows": []}
    cases = {"f64wduo": (lambda: tfhe_amd.params_from_set("STD128Q"), 128, 11),
             "sf2p": (lambda: tfhe_amd.params_from_logq("STD128", False, 23, 0, 0, 1), 1024, 12)}
    for name in args.which.split(","):
        mk, B, probe = cases[name]
        p = mk()
        bsk, ksk = synthetic_keys(p)
        ctx = tfhe_amd.BinFHEContextHIP(p, library=tfhe_amd.capi.TEST_LIB).GPUSetup(bsk, ksk)
        del bsk, ksk
        row = {"kernel": name, "B": B, "probe": probe}
        for rep in range(2):  # alternating
            row.setdefault("default_ms", []).append(timed(ctx, lib, p, B, {}, args.reps, dev, sp, g))
            row.setdefault("probe_ms", []).append(timed(ctx, lib, p, B, {"probe": probe}, args.reps, dev, sp, g))
        row["bound_gain"] = round(1 - min(row["probe_ms"]) / min(row["default_ms"]), 4)
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
        ctx.GPUClean()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
