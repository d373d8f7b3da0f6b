"""Tiled key switch (each packing form, split on / off) against the gather form at three batches;
prints mismatching columns (the check that found the bit_cast miscompile)."""
import sys, numpy as np
sys.path[:0] = ["tfhe-gpu_amd"]
import tfhe_amd
cp = tfhe_amd.params_from_set("STD128")
rs = np.random.default_rng(3)
bsk = rs.integers(0, cp.Q, cp.bsk_words(), dtype=np.uint64)
ksk = rs.integers(0, cp.qKS, cp.ksk_words(), dtype=np.uint64)
ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
for B in (300, 1029, 5000):
    ext = rs.integers(0, cp.Q, (B, cp.N + 1), dtype=np.uint64)
    ctx.set_knobs(ks_tiled_min=0); g = ctx.MKMSwitch(ext, cp.q)
    ctx.set_knobs(ks_tiled_min=1)
    for pk in ("0", "1"):
        for sp in ("1", "4"):
            ctx.set_knobs(ks_pk=int(pk), ks_split=int(sp))
            t = ctx.MKMSwitch(ext, cp.q)
            bad = np.argwhere(t != g)
            print(B, "pk", pk, "split", sp, "mismatches", len(bad), "cols", sorted(set(bad[:, 1].tolist()))[:12], "cts", sorted(set(bad[:, 0].tolist()))[:8], flush=True)
ctx.GPUClean()
