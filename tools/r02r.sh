set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02r
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r02r/std128.log 2>&1 &&
timeout -k 10 300 python3 bench.py --params STD192 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02r/std192.log 2>&1 &&
timeout -k 10 300 python3 bench.py --params STD128Q --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02r/std128q.log 2>&1 &&
timeout -k 10 600 python3 tools/bench_configs.py C2host C3 C4 C5a C5b > gpurun_out/r02r/configs.log 2>&1 &&
timeout -k 10 300 python3 tools/host_path_bench.py --parts 1 > gpurun_out/r02r/host_path.log 2>&1
rc=$?
for f in std128 std192 std128q; do tail -1 gpurun_out/r02r/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'; done
grep -h '^{' gpurun_out/r02r/configs.log gpurun_out/r02r/host_path.log
exit $rc
