#!/bin/bash
# Same-box A/B of library builds on the key switch alone (tools/ks_bench.py, default split), two alternations:
#   TAG=r06ks CFGS="STD128" BATCHES=1024,8192 LIBS="lib/a.so altlib/x/libtfhe_hip_test.so" tools/ks16_ab.sh
set -u
O=gpurun_out/${TAG:-r06ks}; mkdir -p $O
for r in 1 2; do
  for L in ${LIBS:-tfhe-gpu_amd/lib/libtfhe_hip_test.so}; do
    echo "[$(date +%T)] $L $r"
    TFHE_LIB=$L timeout -k 10 200 python3 -u tools/ks_bench.py ${CFGS:-STD128} --batches ${BATCHES:-1024,8192} --reps 10 --splits 32 > $O/ks_$(basename $(dirname $L))_$r.log 2>&1 || exit 1
    grep config $O/ks_$(basename $(dirname $L))_$r.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('   ', d['batch'], d['gather_ms'], d['tiled_split32_ms'], d['equal'])"
  done
done
echo ks16 done
