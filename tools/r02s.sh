# Round 2 re-entry check: full GPU suite + smoke + headline bench on the rebuilt tree.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02s
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02s/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02s/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r02s/bench.log 2>&1
rc=$?
tail -3 gpurun_out/r02s/pytest_gpu.log; tail -2 gpurun_out/r02s/smoke.log; tail -1 gpurun_out/r02s/bench.log
exit $rc
