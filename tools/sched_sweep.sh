#!/bin/bash
# A/B alternative LLVM scheduling strategies for the fast kernel (lib/libtfhe_hip_<strategy>.so).
set -u
export TMPDIR=/tmp
for st in ${STRATS:-default max-ilp iterative-ilp max-memory-clause}; do
  lib=tfhe-gpu_amd/lib/libtfhe_hip_$st.so
  [ "$st" = default ] && lib=tfhe-gpu_amd/lib/libtfhe_hip.so
  TFHE_LIB=$PWD/$lib timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "std128 and kat or eval_acc_parity and fast" > gpurun_out/sched_test_$st.log 2>&1 || { echo "$st parity FAILED"; exit 1; }
  TFHE_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 > gpurun_out/sched_bench_$st.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/sched_bench_$st.log') if l.startswith('{')][-1]); print('$st', d['value'], d['roofline']['kernel_ms'])"
done
