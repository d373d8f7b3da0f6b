#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root via gpurun):
#   1. bench.py                              -> gpurun_out/bench_$TAG.log
#   2. rocprofv3 --kernel-trace --stats      -> gpurun_out/prof_$TAG/ (same command as 1)
#   3. rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / instruction counts / VALU busy + clock in separate passes
#      (no tracing domains) -> gpurun_out/pmc_$TAG.json (copy to profiles/r01_pmc_blind_rotate.json)
# Each GPU step has its own time limit; the chain stops at the first failure.
set -u
TAG=${1:-r01}
ARGS=${2:-}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py $ARGS > gpurun_out/bench_$TAG.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $ARGS > gpurun_out/pmcf_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $ARGS > gpurun_out/pmcw_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmcm_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $ARGS > gpurun_out/pmcm_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmcb_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $ARGS > gpurun_out/pmcb_$TAG.log 2>&1 &&
python3 tools/pmc_summary.py k_blind_rotate gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG gpurun_out/pmc_$TAG.json gpurun_out/pmcm_$TAG gpurun_out/pmcb_$TAG
rc=$?
echo "profile rc=$rc"
tail -2 gpurun_out/bench_$TAG.log
exit $rc
