#!/bin/bash
# L1/L2 behaviour of the blind-rotation kernel (one --pmc pass, no tracing domains).
# Usage: tools/pmc_cache.sh TAG [bench args]   (TFHE_FAST_VARIANT selects the kernel variant)
set -u
TAG=${1:-cache}
shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > gpurun_out/${TAG}.log 2>&1
rc=$?
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "blind_rotate" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{tag} {k:28s} per-launch {sum(v)/len(v):.4g} (n={len(v)})")
PY
exit $rc
