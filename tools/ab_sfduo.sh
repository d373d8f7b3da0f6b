#!/bin/bash
# Same-box A/B of sfduo builds (tools/alt_build.sh variants): the blind rotation at 64 / 128 in C3's context
# (tools/duo_probe.py --ctx ARB12: one / duo / no-hand-off rows) and C5b's 128 (tools/small_batch.py duo2),
# alternating the builds `rounds` times.  GPU box, repo root:  tools/ab_sfduo.sh TAG "LIB_A LIB_B ..." [rounds]
set -u
TAG=$1; LIBS=$2; R=${3:-2}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for L in $LIBS; do
    echo "[$(date +%T)] $L round $r"
    timeout -k 10 200 python3 -u tools/duo_probe.py --ctx ARB12 --lib $L --reps 5 >> $O/arb_probe.log 2>&1 || { echo "rc=$?"; exit 1; }
    timeout -k 10 200 python3 -u tools/small_batch.py duo2 --lib $L --reps 5 >> $O/duo2.log 2>&1 || { echo "rc=$?"; exit 1; }
  done
done
echo "ab_sfduo rc=0"
