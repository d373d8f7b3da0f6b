#!/usr/bin/env python3
"""End-to-end throughput of the drop-in: the reference's unchanged vector
BinFHEContext::EvalBinGate (binfhecontext.cpp:323-325 -> binfhe-base-scheme.cpp:598-677) on the
MI355X through the shim (oracle/_ref/ref_dropin), against the library's host-array API
(tfhe_eval_bin_gate) on the same inputs and keys, in one process pair on one box.

Reports bootstraps/s for both and the shim's per-phase times (TFHE_SHIM_TIMING), so the time
the reference's own host glue takes (copies, BootstrapGateCore's test vectors, extraction --
code the drop-in does not change) is separated from the shim's marshalling and the device.

    python3 tools/dropin_bench.py [B] [reps]
"""
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tfhe-gpu_amd")]
import pyoracle  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ref_dropin")


def main():
    p = pyoracle.params_from_set("STD128")
    c1 = pyoracle.splitmix(pyoracle.Rng(77), B * (p.n + 1), p.q).reshape(B, p.n + 1)
    c2 = pyoracle.splitmix(pyoracle.Rng(78), B * (p.n + 1), p.q).reshape(B, p.n + 1)
    res = {"config": "STD128 EvalBinGate(NAND)", "B": B, "reps": REPS}
    with tempfile.TemporaryDirectory() as tmp:
        f1, f2, fo = (os.path.join(tmp, x) for x in ("c1.bin", "c2.bin", "out.bin"))
        c1.tofile(f1)
        c2.tofile(f2)
        env = dict(os.environ, TFHE_SHIM_TIMING="1")
        r = subprocess.run([DROPIN, "ctx=set:STD128", "keys=synth:1", "op=NAND", "api=vector", "gpus=1",
                            f"in={f1}", f"in2={f2}", f"out={fo}", f"reps={REPS}"],
                           capture_output=True, text=True, env=env, timeout=900)
        if r.returncode:
            sys.exit(r.stderr[-3000:])
        if os.environ.get("DROPIN_STDERR"):  # e.g. with TFHE_TRACE=1: the engine's staging timeline
            open(os.environ["DROPIN_STDERR"], "w").write(r.stderr)
        js = json.loads(r.stdout.strip().splitlines()[-1])
        dropin_out = np.fromfile(fo, dtype=np.uint64).reshape(B, p.n + 1)
    phases = {}
    for m in re.finditer(r"\[shim\] (\w+) (.+?) B=(\d+) ([\d.]+) ms", r.stderr):
        if int(m.group(3)) == B:
            phases.setdefault(f"{m.group(1)} {m.group(2)}", []).append(float(m.group(4)))
    per_rep = {k: min(v) for k, v in phases.items()}
    shim_ms = sum(v for k, v in per_rep.items() if not k.startswith("GPUSetup"))
    res["dropin"] = {"best_s": js["best_s"], "mean_s": js["mean_s"], "bootstraps_per_s": B / js["best_s"],
                     "gpu_setup_s": js.get("gpu_setup_s"), "shim_phase_ms": per_rep,
                     "shim_total_ms": shim_ms, "reference_glue_ms": js["best_s"] * 1e3 - shim_ms}

    import tfhe_amd

    cp = tfhe_amd.params_from_set("STD128")
    bsk, ksk = pyoracle.kat_keys(p, pyoracle.Rng(1))
    ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    best = 1e30
    for _ in range(REPS + 1):
        t = time.perf_counter()
        out = ctx.EvalBinGate("NAND", c1, c2)
        best = min(best, time.perf_counter() - t)
    res["host_array"] = {"best_s": best, "bootstraps_per_s": B / best}
    res["outputs_equal"] = bool(np.array_equal(out, dropin_out))
    res["shim_vs_host_array"] = shim_ms / 1e3 / best
    print(json.dumps(res))


if __name__ == "__main__":
    main()
