set -u
export TMPDIR=/tmp
for v in ${VARS:-0 9 10}; do
  TFHE_TIMING_EXPERIMENTS=1 TFHE_FAST_VARIANT=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 > gpurun_out/exp_$v.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/exp_$v.log') if l.startswith('{')][-1]); print('variant $v kernel_ms', d['roofline']['kernel_ms'])"
done
