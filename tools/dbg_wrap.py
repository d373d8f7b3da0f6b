"""Debug: the STD128Q / STD128Q_OPT WRAP-correction scenario of
tests/test_gpu_parity.py::test_wrap_correction_late_round, repeated on one context: which
ciphertexts differ from the oracle, how many coefficients, and whether two GPU runs on the same
inputs agree with each other (a race shows as run-to-run differences).
Usage: python3 tools/dbg_wrap.py [reps]   (TFHE_LIB selects another build)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tfhe_amd  # noqa: E402
import pyoracle  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
print("lib", os.environ.get("TFHE_LIB", "default"), flush=True)
for pset in ("STD128Q", "STD128Q_OPT"):
    op, cp = pyoracle.params_from_set(pset), tfhe_amd.params_from_set(pset)
    rs = np.random.default_rng(11)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = pyoracle.Oracle(op, bsk, ksk)
    B = 3
    a = np.zeros((B, op.n), dtype=np.uint64)
    a[:, -1] = rs.integers(1, op.q, B, dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    half = op.Q >> 1
    acc[:, :, 10:20] = (half - 1 - rs.integers(0, 1 << 23, (B, 2, 10))).astype(np.uint64)
    acc[2] = rs.integers(0, op.Q, (2, op.N), dtype=np.uint64)
    c = orc.eval_acc(a, op.q, acc)
    prev = None
    for r in range(reps):
        g = ctx.EvalAcc(a, op.q, acc)
        diff = [(b, int((g[b] != c[b]).sum())) for b in range(B) if not np.array_equal(g[b], c[b])]
        self_diff = None if prev is None else int((g != prev).sum())
        prev = g
        print(pset, "kernel", ctx.info().br_kernel, "rep", r, "vs oracle (ct, coeffs)", diff,
              "vs previous run", self_diff, flush=True)
    # the same with a fresh random a (every round active)
    for r in range(2):
        a2 = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
        g = ctx.EvalAcc(a2, op.q, acc)
        c2 = orc.eval_acc(a2, op.q, acc)
        print(pset, "random a rep", r, "vs oracle", [b for b in range(B) if not np.array_equal(g[b], c2[b])], flush=True)
    ctx.GPUClean()
    orc.close()
