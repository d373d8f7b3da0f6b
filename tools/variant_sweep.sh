#!/bin/bash
# A/B the specialised blind-rotation kernel variants (TFHE_FAST_VARIANT) in one box session.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
VARS=${VARS:-"0 1 2 3 4"}
for v in $VARS; do
  TFHE_FAST_VARIANT=$v timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "std128 or fast" > gpurun_out/sweep_test_$v.log 2>&1 || { echo "variant $v: parity FAILED"; tail -5 gpurun_out/sweep_test_$v.log; exit 1; }
  TFHE_FAST_VARIANT=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 > gpurun_out/sweep_bench_$v.log 2>&1 || { echo "variant $v: bench FAILED"; tail -5 gpurun_out/sweep_bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_bench_$v.log').read().strip().splitlines()[-1]); print('variant $v', d['value'], 'bs/s  kernel_ms', d['roofline']['kernel_ms'], 'issue_frac', d['valu'].get('issue_frac'))"
done
