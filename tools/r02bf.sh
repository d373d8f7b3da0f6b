#!/bin/bash
# fast4 (headline) under other LLVM scheduling strategies (altlib/libtfhe_hip_f4_<strategy>.so:
# only blind_rotate_fast4.hip rebuilt with -mllvm -amdgpu-sched-strategy=...): parity, then the
# headline bench alternating with the default build on one box.
set -u
export TMPDIR=/tmp
D=gpurun_out/r02bf
mkdir -p $D
for st in max-ilp iterative-ilp; do
  TFHE_LIB=$PWD/altlib/libtfhe_hip_f4_$st.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "kat or eval_acc or bin_gate" > $D/pytest_$st.log 2>&1 || { echo "$st parity FAILED"; tail -20 $D/pytest_$st.log; exit 1; }
  echo "$st $(tail -1 $D/pytest_$st.log)"
done
for rep in 1 2 3; do
  for st in default max-ilp iterative-ilp; do
    L=""; [ $st != default ] && L="TFHE_LIB=$PWD/altlib/libtfhe_hip_f4_$st.so"
    env $L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $D/${st}_$rep.log 2>&1 || { tail -5 $D/${st}_$rep.log; exit 1; }
    echo "STD128 $st rep=$rep $(tail -1 $D/${st}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
