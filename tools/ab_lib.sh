#!/bin/bash
# Same-box A/B of library builds on the device-resident bench (run on the GPU box from the repo root):
#   tools/ab_lib.sh TAG "C3 C5b" "LIB_A LIB_B [LIB_C ...]" [rounds] [extra bench args, e.g. "--batch 128"]
# alternates the builds per configuration, `rounds` times (bench.py without CPU baseline / host array /
# drop-in legs; TFHE_LIB selects the build); one JSON line per run -> gpurun_out/$TAG/ab_CFG_<i>_<round>.log
set -u
TAG=$1; CFGS=$2; LIBS=$3; R=${4:-2}; EXTRA=${5:-}; SFX=${EXTRA// /}
O=gpurun_out/$TAG
mkdir -p $O
for CFG in $CFGS; do
  for r in $(seq 1 $R); do
    i=0
    for L in $LIBS; do
      i=$((i + 1))
      echo "[$(date +%T)] $CFG lib$i round $r ($L)"
      TFHE_ABI_PREV=1 TFHE_LIB=$L timeout -k 10 300 python3 bench.py --config $CFG --no-cpu-baseline --no-host-array --no-dropin \
        --steps 3 --warmup 1 $EXTRA > $O/ab_${CFG}${SFX}_${i}_$r.log 2>&1 || { echo "ab rc=$?"; exit 1; }
      tail -1 $O/ab_${CFG}${SFX}_${i}_$r.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('   ', l['value'], 'kernel_ms', r['kernel_ms'])"
    done
  done
done
echo "ab rc=0"
