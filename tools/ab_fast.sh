#!/bin/bash
# A/B of specialised-kernel builds (TFHE_FAST_VARIANT) on one box: parity of every build, then
# alternating device-resident bench reps.  Usage (via gpurun): bash tools/ab_fast.sh TAG "60 61 62" [reps]
set -u
TAG=$1; VARS=$2; REPS=${3:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernel_variants.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -20 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for r in $(seq 1 $REPS); do
  for v in $VARS; do
    TFHE_FAST_VARIANT=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dropin --no-host-array --steps 10 > gpurun_out/$TAG/bench_${v}_$r.log 2>&1 || { tail -5 gpurun_out/$TAG/bench_${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/$TAG/bench_${v}_$r.log') if l.startswith('{')][-1]); print('variant $v rep $r', d['value'], d['roofline']['kernel_ms'])" | tee -a gpurun_out/$TAG/summary.txt
  done
done
