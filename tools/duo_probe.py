#!/usr/bin/env python3
"""What the per-round hand-off costs the two-workgroup blind rotations (f64wduo: C5a's 8-GPU shard; sfduo<1>:
C3's context at small batches, --ctx ARB12).

Test library (lib/libtfhe_hip_test.so, or --lib): STD128Q, device-resident blind rotation at B = 64 / 128, timed
(min of --reps, HIP stream sync) for
  one   f64w, one workgroup per ciphertext (duo = 0)
  duo   f64wduo (the default for B <= 128)
  free  f64wduo with NO hand-off (probe 7: each member takes its own stage-1 values for its partner's;
        results invalid) -- the lower bound of the duo form, i.e. the exchange's price per round.
  bcast f64wduo with wave-uniform monomial-factor rows (probe 9, results invalid): what the factor
        tables' LDS bank conflicts cost.
--ctx ARB12: the same one / duo / free rows for sfduo<1> (probe 7 there too).
One JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-gpu_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ctx", default="STD128Q", choices=["STD128Q", "ARB12"])
    ap.add_argument("--lib", default=None, help="a test-library build (default lib/libtfhe_hip_test.so)")
    args = ap.parse_args()
    import torch

    import tfhe_amd
    from bench import synthetic_keys

    p = (tfhe_amd.params_from_set("STD128Q") if args.ctx == "STD128Q"
         else tfhe_amd.params_from_logq("STD128", True, 12, 0, 0, 1))
    bsk, ksk = synthetic_keys(p)
    libpath = args.lib or tfhe_amd.capi.TEST_LIB
    ctx = tfhe_amd.BinFHEContextHIP(p, library=libpath).GPUSetup(bsk, ksk)
    del bsk, ksk
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    lib = ctx._L
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    rows = []
    for B in (64, 128):
        a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
        acc0 = torch.randint(0, int(p.Q), (B, 2, p.N), dtype=torch.int64, device=dev, generator=g)
        row = {"B": B}
        forms = [("one", {"duo": 0}), ("duo", {}), ("free", {"probe": 7})]
        if args.ctx == "STD128Q":
            forms.append(("bcast", {"probe": 9}))
        for tag, knobs in forms:
            acc = acc0.clone()
            with ctx.knobs_set(**knobs):
                ts = []
                for _ in range(args.reps + 1):
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    tfhe_amd.capi.check(lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp),
                                        "eval_acc")
                    torch.cuda.synchronize(dev)
                    ts.append(time.perf_counter() - t0)
            finals = row.setdefault("_finals", {})
            finals[tag] = acc.cpu()
            row[f"{tag}_ms"] = round(min(ts[1:]) * 1e3, 3)
            row[f"{tag}_us_per_round"] = round(min(ts[1:]) * 1e6 / p.n, 2)
        row["handoff_us_per_round"] = round(row["duo_us_per_round"] - row["free_us_per_round"], 2)
        finals = row.pop("_finals")
        row["duo_equals_one"] = bool(torch.equal(finals["duo"], finals["one"]))  # same inputs, same number of runs
        rows.append(row)
    kern = "f64wduo" if args.ctx == "STD128Q" else "sfduo<1>"
    print(json.dumps({"what": f"{kern} hand-off price ({args.ctx} blind rotation, device-resident)", "lib": libpath,
                      "rows": rows}), flush=True)
    ctx.GPUClean()


if __name__ == "__main__":
    main()
