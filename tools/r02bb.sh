#!/bin/bash
# Wave-cycle split (parked / issue-stalled / issuing) and LDS conflicts of the blind-rotation
# kernels: headline STD128 (fast4), STD192 and STD128Q (f64w).  One --pmc pass per set.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02bb
rc=0
for ps in STD128 STD192 STD128Q; do
  CMD="python3 bench.py --params $ps --no-cpu-baseline --steps 1 --warmup 0" timeout -k 10 240 bash tools/pmc_wait.sh r02bb/wait_$ps > gpurun_out/r02bb/wait_$ps.txt 2>&1 || { rc=1; break; }
  echo "$ps: $(cat gpurun_out/r02bb/wait_$ps.txt)"
done
exit $rc
