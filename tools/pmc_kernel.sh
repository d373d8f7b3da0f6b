#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, no tracing domains) over any command,
# summarised per launch for the kernels whose name contains FILTER.
# Usage: tools/pmc_kernel.sh FILTER TAG cmd args...
set -u
FILTER=$1
TAG=$2
shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
  "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
)
rc=0
k=0
for g in "${groups[@]}"; do
  timeout -s KILL 200 rocprofv3 --pmc $g -d gpurun_out/${TAG}_p$k -o run --output-format csv -- "$@" > gpurun_out/${TAG}_p$k.log 2>&1 || { rc=$?; break; }
  k=$((k+1))
done
python3 - "$TAG" "$FILTER" <<'PY'
import csv, glob, sys, collections
tag, flt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/{tag}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:24s} per-launch {sum(v)/len(v):.4g} (n={len(v)})")
PY
exit $rc
