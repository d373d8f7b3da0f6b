#!/usr/bin/env python3
"""Repeated-call soak of the blind rotation (device-resident EvalAcc) per kernel family: the same
inputs R times at a full batch; every call's output must equal the first call's bit for bit, and the
first call's first ciphertexts must equal the oracle.  Evidence that no intermittent wrong-result
hazard (the round-2 f64w race) remains on the default kernels.
Usage: python3 tools/soak.py [STD128:300 STD128Q:30 STD192:30 LOGQ23:30] [--batch 8192]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tfhe-gpu_amd"), os.path.join(ROOT, "oracle")]

SETS = {
    "STD128": lambda m: m.params_from_set("STD128"),
    "STD128Q": lambda m: m.params_from_set("STD128Q"),
    "STD192": lambda m: m.params_from_set("STD192"),
    "LOGQ23": lambda m: m.params_from_logq("STD128", False, 23, 0, 0, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("runs", nargs="*", default=["STD128:300", "STD128Q:30", "STD192:30", "LOGQ23:30"])
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--check", type=int, default=4, help="ciphertexts of the first call checked by the oracle")
    args = ap.parse_args()
    import torch

    import pyoracle
    import tfhe_amd
    from tfhe_amd import capi

    for spec in args.runs:
        name, reps = spec.split(":")
        reps, B = int(reps), args.batch
        p, op = SETS[name](tfhe_amd), SETS[name](pyoracle)
        rs = np.random.default_rng(7)
        bsk = rs.integers(0, p.Q, p.bsk_words(), dtype=np.uint64)
        ksk = rs.integers(0, p.qKS, p.ksk_words(), dtype=np.uint64)
        ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
        a = rs.integers(0, p.q, (B, p.n), dtype=np.uint64)
        acc = rs.integers(0, p.Q, (B, 2, p.N), dtype=np.uint64)
        da = torch.from_numpy(a.view(np.int64)).cuda()
        dacc0 = torch.from_numpy(acc.view(np.int64)).cuda()
        dacc = torch.empty_like(dacc0)
        s = torch.cuda.Stream()
        first, bad = None, 0
        t0 = time.perf_counter()
        for r in range(reps):
            dacc.copy_(dacc0)
            torch.cuda.synchronize()
            capi.check(capi.lib().tfhe_eval_acc_device(ctx.handle, B, da.data_ptr(), int(p.q), dacc.data_ptr(),
                                                       s.cuda_stream), "eval_acc_device")
            s.synchronize()
            out = dacc.cpu().numpy().view(np.uint64)
            if first is None:
                first = out.copy()
            elif not np.array_equal(out, first):
                bad += int((out != first).reshape(B, -1).any(axis=1).sum())
        dt = time.perf_counter() - t0
        orc = pyoracle.Oracle(op, bsk, ksk)
        k = args.check
        ref = orc.eval_acc(np.ascontiguousarray(a[:k]), p.q, np.ascontiguousarray(acc[:k]))
        orc.close()
        res = {"set": name, "batch": B, "calls": reps, "kernel": ctx.info().br_kernel,
               "wrong_ciphertexts_vs_first_call": bad, "oracle_checked": k,
               "oracle_bit_exact": bool(np.array_equal(ref, first[:k])), "seconds": round(dt, 1)}
        print(json.dumps(res), flush=True)
        ctx.GPUClean()


if __name__ == "__main__":
    main()
