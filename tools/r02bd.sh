#!/bin/bash
# Host-array configurations C2host..C5b (tools/bench_configs.py) on the final round-2 tree.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02bd
timeout -k 10 900 python3 -u tools/bench_configs.py C2host C3 C4 C5a C5b > gpurun_out/r02bd/configs.log 2>&1
rc=$?
grep -h '^{' gpurun_out/r02bd/configs.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], d['bootstraps_per_s'])"
exit $rc
