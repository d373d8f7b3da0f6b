#!/bin/bash
# PMC passes of one configuration's blind rotation for several library builds (run on the GPU box):
#   tools/pmc_ab.sh TAG CFG "LIB_A LIB_B ..."
# per build: FETCH_SIZE; TCC_HIT_sum TCC_MISS_sum; SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES
# (one counter group per run, no tracing domains) -> gpurun_out/$TAG/pmcab_CFG_<i>.json
set -u
TAG=$1; CFG=$2; LIBS=$3
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
Q="--config $CFG --no-cpu-baseline --no-host-array --no-dropin --steps 1 --warmup 1 --kernel-reps 1"
i=0
for L in $LIBS; do
  i=$((i + 1))
  echo "[$(date +%T)] $CFG lib$i $L"
  for g in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"; do
    n=$(echo $g | cut -c1-8)
    TFHE_ABI_PREV=1 TFHE_LIB=$L timeout -s KILL 300 rocprofv3 --pmc $g -d $O/pab_${CFG}_${i}_$n -o run --output-format csv -- \
      python3 bench.py $Q > $O/pab_${CFG}_${i}_$n.log 2>&1 || { echo "pmc_ab rc=$?"; exit 1; }
  done
  python3 tools/pmc_counters.py k_blind_rotate $O/pab_${CFG}_${i}_* > $O/pmcab_${CFG}_$i.json
  echo "   $(cat $O/pmcab_${CFG}_$i.json)"
done
echo "pmc_ab rc=0"
