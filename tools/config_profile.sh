#!/bin/bash
# One SURVEY 8(d) configuration measured like the headline (run on the GPU box from the repo root):
#   1. bench.py --config CFG (device-resident value, roofline vs the matching VALU peak, reference CPU
#      baseline on the same context, keys and inputs)                  -> gpurun_out/$TAG/bench_CFG.log
#   2. rocprofv3 --kernel-trace --stats of the same command (no CPU leg) -> gpurun_out/$TAG/prof_CFG/
#   3. PMC passes on the blind rotation (FETCH_SIZE, WRITE_SIZE, instruction mix, VALU busy + clock),
#      one counter group per run, no tracing domains                  -> gpurun_out/$TAG/pmc_CFG.json
#   4. bench.py --config CFG again, now reading that PMC record (busy fraction, held clock, traffic)
# Usage: tools/config_profile.sh TAG "C3 C4 C5a C5b" [extra bench args]
set -u
TAG=$1
CFGS=$2
EXTRA=${3:-}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
rc=0
for CFG in $CFGS; do
  case $CFG in C2) B=8192 ;; C3) B=4096 ;; C4) B=8192 ;; C5a|C5b) B=1024 ;; *) echo "unknown $CFG"; exit 2 ;; esac
  Q="--config $CFG --no-cpu-baseline --no-host-array --no-dropin --steps 1 --warmup 1 --kernel-reps 1 $EXTRA"
  echo "[$(date +%T)] $CFG rocprof" &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$CFG -o run --output-format csv -- python3 bench.py --config $CFG --no-cpu-baseline --no-dropin $EXTRA > $O/prof_$CFG.log 2>&1 &&
  echo "[$(date +%T)] $CFG pmc" &&
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_$CFG -o run --output-format csv -- python3 bench.py $Q > $O/pmcf_$CFG.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$CFG -o run --output-format csv -- python3 bench.py $Q > $O/pmcw_$CFG.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT -d $O/pmcm_$CFG -o run --output-format csv -- python3 bench.py $Q > $O/pmcm_$CFG.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmcb_$CFG -o run --output-format csv -- python3 bench.py $Q > $O/pmcb_$CFG.log 2>&1 &&
  PMC_UNITS=$B python3 tools/pmc_summary.py k_blind_rotate $O/pmcf_$CFG $O/pmcw_$CFG $O/pmc_$CFG.json $O/pmcm_$CFG $O/pmcb_$CFG > /dev/null &&
  echo "[$(date +%T)] $CFG bench" &&
  timeout -k 10 900 python3 bench.py --config $CFG --pmc-json $O/pmc_$CFG.json $EXTRA > $O/bench_$CFG.log 2>&1 || { rc=$?; break; }
  tail -1 $O/bench_$CFG.log | cut -c1-300
done
echo "config_profile rc=$rc"
exit $rc
