#!/bin/bash
# iterative-ilp for the special-form / generic kernels (altlib/libtfhe_hip_gen_ilp.so: C3, C5b)
# and for the tiled key switch (altlib/libtfhe_hip_ks_ilp.so: headline step), against the tree
# build, alternating on one box; parity first.  (Not yet run: rebuild the two altlib/ files from
# the tree objects with the one translation unit recompiled under -mllvm -amdgpu-sched-strategy=iterative-ilp.)
set -u
export TMPDIR=/tmp
D=gpurun_out/r02bi
mkdir -p $D
TFHE_LIB=$PWD/altlib/libtfhe_hip_gen_ilp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "logq or n2048" > $D/pytest_gen.log 2>&1 || { echo "gen parity FAILED"; tail -20 $D/pytest_gen.log; exit 1; }
echo "gen $(tail -1 $D/pytest_gen.log)"
TFHE_LIB=$PWD/altlib/libtfhe_hip_ks_ilp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_keyswitch.py -x -q --timeout 120 --timeout-method thread > $D/pytest_ks.log 2>&1 || { echo "ks parity FAILED"; tail -20 $D/pytest_ks.log; exit 1; }
echo "ks $(tail -1 $D/pytest_ks.log)"
for rep in 1 2; do
  for st in tree gen_ilp; do
    L=""; [ $st != tree ] && L="TFHE_LIB=$PWD/altlib/libtfhe_hip_$st.so"
    env $L timeout -k 10 300 python3 -u tools/bench_configs.py C3 C5b > $D/cfg_${st}_$rep.log 2>&1 || { tail -5 $D/cfg_${st}_$rep.log; exit 1; }
    grep -h '^{' $D/cfg_${st}_$rep.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], '$st', $rep, d['bootstraps_per_s'])"
  done
  for st in tree ks_ilp; do
    L=""; [ $st != tree ] && L="TFHE_LIB=$PWD/altlib/libtfhe_hip_$st.so"
    env $L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $D/c2_${st}_$rep.log 2>&1 || { tail -5 $D/c2_${st}_$rep.log; exit 1; }
    echo "STD128 $st $rep $(tail -1 $D/c2_${st}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
