#!/bin/bash
# Round-4 measurement pass on the GPU box (from the repo root via gpurun):
#   1. VALU peaks of every product the blind rotations issue (valu_rates) + a GRBM_GUI_ACTIVE pass
#      for the clock held under each  -> gpurun_out/$TAG/valu_rates.txt, valu_peak.json
#   2. the new device-resident entry points' GPU tests
#   3. small-batch sweeps (tools/small_batch.py: C5 EvalSign 128..1024, CHES AND 256 x 1000, CHES EvalFunc)
# Each GPU step has its own time limit; the chain stops at the first failure.
set -u
TAG=${1:-r04a}
STEPS=${2:-"peak tests small"}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
rc=0
for s in $STEPS; do
  case $s in
    peak)
      timeout -k 10 120 tools/microbench/valu_rates > $O/valu_rates.txt 2>&1 &&
      timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/valu_pmc -o run --output-format csv -- tools/microbench/valu_rates > $O/valu_pmc.log 2>&1 &&
      python3 tools/valu_peak.py $O/valu_rates.txt $O/valu_pmc > $O/valu_peak.json || rc=$? ;;
    tests)
      timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gpu_device_ops.py tests/test_gpu_c5.py > $O/pytest_new.log 2>&1 || rc=$? ;;
    small)
      timeout -k 10 900 python3 -u tools/small_batch.py sign and func > $O/small_batch.log 2>&1 || rc=$? ;;
    ks)
      timeout -k 10 600 python3 -u tools/ks_bench.py STD128Q LOGQ23 STD192 ARB12 STD128 --reps 5 \
        --batches 1,4,16,64,128,256,512,1024 --splits 4,16 > $O/ks_sweep.log 2>&1 || rc=$? ;;
    suite)
      # the whole GPU suite under a kernel trace: which kernel instances the parity tests run
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/suite_prof -o run --output-format csv -- \
        python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || rc=$? ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || rc=$? ;;
    *)
      echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -ne 0 ] && break
done
echo "measure rc=$rc"
exit $rc
