#!/bin/bash
# Issue/stall counters of the blind-rotation kernel (separate --pmc passes, no tracing domains).
# Usage: tools/pmc_stall.sh TAG [bench args]
set -u
TAG=${1:-stall}
shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${CMD:-"python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $*"}
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU2 SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_IFETCH GRBM_GUI_ACTIVE -d gpurun_out/${TAG}_a -o run --output-format csv -- $B > gpurun_out/${TAG}_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES -d gpurun_out/${TAG}_b -o run --output-format csv -- $B > gpurun_out/${TAG}_b.log 2>&1
rc=$?
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
for part in "ab":
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/{tag}_{part}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "blind_rotate" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{part} {k:24s} per-launch {sum(v)/len(v):.4g} (n={len(v)})")
PY
exit $rc
