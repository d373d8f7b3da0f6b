# Full GPU suite + smoke + headline bench + every SURVEY 8(d) configuration on the current tree.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02af
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02af/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02af/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02af/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02af/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r02af/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --params STD192 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02af/std192.log 2>&1 &&
timeout -k 10 300 python3 bench.py --params STD128Q --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02af/std128q.log 2>&1 &&
timeout -k 10 700 python3 tools/bench_configs.py C2host C3 C4 C5a C5b > gpurun_out/r02af/configs.log 2>&1
rc=$?
tail -1 gpurun_out/r02af/smoke.log
for f in bench std192 std128q; do tail -1 gpurun_out/r02af/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"], d["value"], d["roofline"]["kernel_ms"])'; done
grep -h '^{' gpurun_out/r02af/configs.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], d['kernel'], d['bootstraps_per_s'])"
exit $rc
