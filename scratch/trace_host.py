"""One traced host-array NAND (B = 8192) and one traced EvalAcc: where the host-array time goes."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tfhe-gpu_amd"), ROOT]
import tfhe_amd
from bench import synthetic_keys
cp = tfhe_amd.params_from_set("STD128")
bsk, ksk = synthetic_keys(cp)
ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
rs = np.random.default_rng(1)
B = 8192
c1 = rs.integers(0, cp.q, (B, cp.n + 1), dtype=np.uint64)
c2 = rs.integers(0, cp.q, (B, cp.n + 1), dtype=np.uint64)
for r in range(3):
    t = time.perf_counter(); ctx.EvalBinGate("NAND", c1, c2); print("gate", r, (time.perf_counter() - t) * 1e3, "ms", flush=True)
a = rs.integers(0, cp.q, (B, cp.n), dtype=np.uint64)
acc = np.zeros((B, 2, cp.N), dtype=np.uint64)
acc[:, 1, ::2] = rs.integers(0, cp.Q, (B, cp.N // 2), dtype=np.uint64)
for r in range(3):
    t = time.perf_counter(); ctx.EvalAcc(a, cp.q, acc); print("evalacc", r, (time.perf_counter() - t) * 1e3, "ms", flush=True)
ctx.GPUClean()
