#!/bin/bash
# Same-box A/B of library builds on the blind rotation alone (tools/br_ab.py), alternating `rounds` times:
#   tools/br_ab.sh TAG CTX BATCHES "LIB_A LIB_B ..." [rounds]      (a LIB of "default" = the product library)
set -u
TAG=$1; CTX=$2; BATCHES=$3; LIBS=$4; R=${5:-2}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for L in $LIBS; do
    echo "[$(date +%T)] $L round $r"
    if [ "$L" = default ]; then A=""; else A="--lib $L"; fi
    timeout -k 10 300 python3 -u tools/br_ab.py --ctx $CTX --batches $BATCHES --reps 5 $A >> $O/br_ab.log 2>&1 || { echo "rc=$?"; exit 1; }
    tail -1 $O/br_ab.log
  done
done
echo "br_ab rc=0"
