"""Timeline of the host-array EvalAcc (flat and rows) at B=8192 with TFHE_TRACE=1 (stderr)."""
import ctypes as C, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tfhe-gpu_amd")]
import tfhe_amd
from tfhe_amd.capi import check
cp = tfhe_amd.params_from_set("STD128")
rs = np.random.default_rng(1)
bsk = rs.integers(0, cp.Q, cp.bsk_words(), dtype=np.uint64)
ksk = rs.integers(0, cp.qKS, cp.ksk_words(), dtype=np.uint64)
ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
lib = tfhe_amd.lib()
B, amod, tvlen = 8192, cp.q, cp.q // 2
a = rs.integers(0, amod, (B, cp.n), dtype=np.uint64)
tv = rs.integers(0, cp.Q, (B, tvlen), dtype=np.uint64)
flat = np.empty((B, 2, cp.N), dtype=np.uint64)
a_rows = [np.array(x) for x in a]
acc_rows = [np.empty(cp.N, dtype=np.uint64) for _ in range(2 * B)]
P = lambda arrs: (C.c_void_p * len(arrs))(*[x.ctypes.data for x in arrs])
pa, pc = P(a_rows), P(acc_rows)
for rep in range(3):
    for kind in ("flat", "rows"):
        sys.stderr.write(f"--- {kind} rep {rep}\n"); sys.stderr.flush()
        t = time.perf_counter()
        if kind == "flat":
            check(lib.tfhe_eval_acc_tv(ctx.handle, B, a, amod, tv, tvlen, flat), "acc_tv")
        else:
            check(lib.tfhe_eval_acc_tv_rows(ctx.handle, B, pa, amod, tv, tvlen, pc), "acc_tv_rows")
        sys.stderr.write(f"--- {kind} rep {rep}: {1e3 * (time.perf_counter() - t):.2f} ms\n"); sys.stderr.flush()
ctx.GPUClean()
