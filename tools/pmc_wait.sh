#!/bin/bash
# Wave-cycle split of the blind-rotation kernel: parked (s_waitcnt / barrier), issue-stalled,
# issuing (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES), plus LDS
# instruction and bank-conflict counts.  One --pmc pass, no tracing domains.
# Usage: CMD="python3 bench.py ..." tools/pmc_wait.sh TAG
set -u
TAG=${1:-wait}
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${CMD:-"python3 bench.py --no-cpu-baseline --steps 1 --warmup 0"}
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d gpurun_out/${TAG} -o run --output-format csv -- $B > gpurun_out/${TAG}.log 2>&1
rc=$?
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
for f in glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f)):
        if "blind_rotate" in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"][:60]
    for d, c in agg.items():
        w = c["SQ_WAVE_CYCLES"] or 1
        print(name[d], f"parked {c['SQ_WAIT_ANY']/w:.3f} stalled {c['SQ_WAIT_INST_ANY']/w:.3f} issuing {c['SQ_ACTIVE_INST_ANY']/w:.3f}",
              f"VALU/LDS instr {c['SQ_INSTS_VALU']/max(c['SQ_INSTS_LDS'],1):.1f} bank-conflict/LDS-instr {c['SQ_LDS_BANK_CONFLICT']/max(c['SQ_INSTS_LDS'],1):.2f}")
PY
exit $rc
