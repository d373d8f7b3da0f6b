"""Debug: repeated EvalAcc parity (new random inputs each time) on STD192 (f64w) and the logQ = 12
arbFunc context (sf2, one digit); prints the ciphertexts that differ from the oracle.
Usage: python3 tools/dbg_ct0.py [reps] [STD192 arb12 logq23 STD128Q ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tfhe_amd  # noqa: E402
import pyoracle  # noqa: E402
from tfhe_amd import capi  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
names = sys.argv[2:] or ["STD192", "arb12"]
for name in names:
    if name == "arb12":
        op, cp = pyoracle.params_from_logq("STD128", True, 12, 0, 0, 1), capi.params_from_logq("STD128", True, 12, 0, 0, 1)
    elif name == "logq23":  # C5b: sf2 with two digits
        op, cp = pyoracle.params_from_logq("STD128", False, 23, 0, 0, 1), capi.params_from_logq("STD128", False, 23, 0, 0, 1)
    else:
        op, cp = pyoracle.params_from_set(name), capi.params_from_set(name)
    rs = np.random.default_rng(5)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = pyoracle.Oracle(op, bsk, ksk)
    bad = 0
    for r in range(reps):
        B = 4
        a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
        acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
        g = ctx.EvalAcc(a, op.q, acc)
        c = orc.eval_acc(a, op.q, acc)
        diff = [b for b in range(B) if not np.array_equal(g[b], c[b])]
        bad += bool(diff)
        print(name, "kernel", ctx.info().br_kernel, "rep", r, "differing ciphertexts", diff, flush=True)
    print(name, "reps with a difference:", bad, "of", reps, flush=True)
    ctx.GPUClean()
    orc.close()
