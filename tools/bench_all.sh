#!/bin/bash
# Every SURVEY 8(d) configuration through bench.py on one GPU box (run from the repo root): the full
# JSON line per configuration (device-resident value, roofline against the matching VALU peak
# profiles/r04_valu_peak.json, the per-config PMC record profiles/r04_pmc_CFG.json, the reference's
# CPU baseline on the same context, keys and inputs)  -> gpurun_out/$TAG/bench_CFG.log
set -u
TAG=$1; CFGS=${2:-"C2 C3 C4 C5a C5b"}
O=gpurun_out/$TAG
mkdir -p $O
for CFG in $CFGS; do
  echo "[$(date +%T)] $CFG"
  timeout -k 10 600 python3 bench.py --config $CFG > $O/bench_$CFG.log 2>&1 || { echo "bench_all rc=$?"; exit 1; }
  tail -1 $O/bench_$CFG.log | cut -c1-200
done
echo "bench_all rc=0"
