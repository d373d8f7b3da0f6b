# LDS monomial tables in the exact-FP64 kernel: parity (N = 2048 / 1024 sets, WRAP, KATs), then
# STD192 / STD128Q device-resident and C4 / C5a host-array throughput.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ab
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paramsets.py -x -v --timeout 120 --timeout-method thread -k "n2048 or wrap or custom_modulus or kat or paramset" > gpurun_out/r02ab/pytest.log 2>&1
rc=$?
tail -4 gpurun_out/r02ab/pytest.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --params STD192 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02ab/std192.log 2>&1 &&
timeout -k 10 300 python3 bench.py --params STD128Q --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02ab/std128q.log 2>&1 &&
timeout -k 10 500 python3 tools/bench_configs.py C4 C5a > gpurun_out/r02ab/configs.log 2>&1
rc=$?
for f in std192 std128q; do tail -1 gpurun_out/r02ab/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"], d["value"], d["roofline"]["kernel_ms"])'; done
grep -h '^{' gpurun_out/r02ab/configs.log | cut -c1-60,300-420
exit $rc
