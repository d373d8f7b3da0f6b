#!/bin/bash
# GPU-box validation recipe: GPU test suite, smoke(), bench line, rocprofv3 kernel stats.
# Usage (via gpurun, from the repo root): bash tools/validate.sh TAG
set -u
TAG=${1:-val}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/$TAG/prof.log 2>&1
rc=$?
echo "validate rc=$rc"
tail -3 gpurun_out/$TAG/pytest_gpu.log
tail -1 gpurun_out/$TAG/bench.log
exit $rc
