#!/bin/bash
# Same-box A/B of library builds on the key switch alone (tools/ks_bench.py, tiled form at the engine's default
# split, ks40 = 1), alternating the builds `rounds` times.  GPU box, repo root:
#   tools/ks_ab.sh TAG "LIB_A LIB_B ..." "ARB12 LOGQ23" "128,1024,4096" [rounds]
set -u
TAG=$1; LIBS=$2; CFGS=$3; BATCHES=$4; R=${5:-2}
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $R); do
  for L in $LIBS; do
    n=$(basename $(dirname $L))
    echo "[$(date +%T)] $n round $r"
    TFHE_ABI_PREV=1 TFHE_LIB=$L timeout -k 10 300 python3 tools/ks_bench.py $CFGS --batches $BATCHES --reps 5 --ks40 1 \
      > $O/ks_${n}_$r.log 2>&1 || { echo "ks_ab rc=$?"; exit 1; }
    grep config $O/ks_${n}_$r.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); k = [x for x in d if x.startswith('tiled')][0]
    print('   ', d['config'], d['batch'], k, d[k], d['equal'])"
  done
done
echo "ks_ab rc=0"
