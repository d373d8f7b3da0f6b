#!/bin/bash
# STD192 at small batches: the two-workgroup form (f64wduo<0, false, false, 2>, round 6) against the one-workgroup
# f64w (knob duo = 0), device-resident NAND, two alternating reps per batch (GPU box, repo root):
#   tools/duo192.sh TAG
set -u
O=gpurun_out/$1
mkdir -p $O
for B in 64 128; do
  for r in 1 2; do
    for k in 128 0; do
      timeout -k 10 200 python3 bench.py --params STD192 --batch $B --steps 5 --warmup 1 --no-host-array --knob duo=$k \
        > $O/std192_B${B}_duo${k}_$r.log 2>&1 || { echo "rc=$?"; exit 1; }
      tail -1 $O/std192_B${B}_duo${k}_$r.log | python3 -c "
import json, sys
l = json.loads(sys.stdin.read()); r = l['roofline']
print('B=$B duo=$k rep $r', l['value'], 'bootstraps/s, blind rotation', r['kernel_ms'], 'ms')"
    done
  done
done
echo "duo192 rc=0"
