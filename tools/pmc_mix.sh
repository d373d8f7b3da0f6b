#!/bin/bash
# Instruction-mix / stall counters for the blind-rotation kernel (separate --pmc passes,
# no tracing domains).  Usage: tools/pmc_mix.sh TAG [bench args]
set -u
TAG=${1:-mix}
shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${CMD:-"python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $*"}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM -d gpurun_out/${TAG}_a -o run --output-format csv -- $B > gpurun_out/${TAG}_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d gpurun_out/${TAG}_b -o run --output-format csv -- $B > gpurun_out/${TAG}_b.log 2>&1
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
