import sys, time, numpy as np
sys.path.insert(0,'oracle'); sys.path.insert(0,'tfhe-gpu_amd')
import pyoracle as oracle, tfhe_amd as capi
op = oracle.params_from_logq("STD128", True, 12, 0, 0, 1)
cp = capi.params_from_logq("STD128", True, 12, 0, 0, 1)
bsk, ksk = oracle.kat_keys(op, oracle.Rng(51))
ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
rs = np.random.default_rng(8)
ct = rs.integers(0, op.qKS, (1024, op.n + 1), dtype=np.uint64)
mat = rs.integers(0, 64, (1024, 1024), dtype=np.int64)
for i in range(3):
    t=time.time(); out = ctx.CiphertextMulMatrix(ct, mat, op.qKS); print("GEMM.cpp config 1024x1024, n=1305: %.2f ms" % ((time.time()-t)*1e3))
