#!/bin/bash
# The other fast4 digit shapes: tree build (fast4 under iterative-ilp) vs the previous default build
# (altlib/libtfhe_hip_prev.so): EvalFloor logQ = 11 contexts (F11: thrown digit, F11t0: folded) and STD128_AP.
set -u
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r02bg}
mkdir -p $D
for rep in 1 2; do
  for st in prev iterative-ilp; do
    L=""; [ $st = prev ] && L="TFHE_LIB=$PWD/altlib/libtfhe_hip_prev.so"
    env $L timeout -k 10 300 python3 -u tools/bench_configs.py F11 F11t0 > $D/cfg_${st}_$rep.log 2>&1 || { tail -5 $D/cfg_${st}_$rep.log; exit 1; }
    grep -h '^{' $D/cfg_${st}_$rep.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], '$st', $rep, d['bootstraps_per_s'])"
    env $L timeout -k 10 300 python3 bench.py --params STD128_AP --no-cpu-baseline --steps 3 --warmup 1 > $D/ap_${st}_$rep.log 2>&1 || { tail -5 $D/ap_${st}_$rep.log; exit 1; }
    echo "STD128_AP $st $rep $(tail -1 $D/ap_${st}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    env $L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $D/c2_${st}_$rep.log 2>&1 || { tail -5 $D/c2_${st}_$rep.log; exit 1; }
    echo "STD128 $st $rep $(tail -1 $D/c2_${st}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
