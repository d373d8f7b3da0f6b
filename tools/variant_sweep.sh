#!/bin/bash
# A/B the specialised blind-rotation kernel variants (TFHE_FAST_VARIANT) in one box session:
# parity subset first, then the bench; stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
VARS=${VARS:-"34 0"}
TAG=${TAG:-sweep}
for v in $VARS; do
  [ -z "${NOTEST:-}" ] && { TFHE_FAST_VARIANT=$v timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "std128 or fast" > gpurun_out/${TAG}_test_$v.log 2>&1 || { echo "variant $v: parity FAILED"; tail -15 gpurun_out/${TAG}_test_$v.log; exit 1; }; }
  TFHE_FAST_VARIANT=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 > gpurun_out/${TAG}_bench_$v.log 2>&1 || { echo "variant $v: bench FAILED"; tail -5 gpurun_out/${TAG}_bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_bench_$v.log').read().strip().splitlines()[-1]); print('variant $v', d['value'], 'bs/s  kernel_ms', d['roofline']['kernel_ms'])"
done
