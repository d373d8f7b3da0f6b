# LDS monomial tables in the special-form kernels: parity, then C3/C5b throughput.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02aa
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "logq or kat or floor_sign" > gpurun_out/r02aa/pytest.log 2>&1
rc=$?
tail -4 gpurun_out/r02aa/pytest.log
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python3 tools/bench_configs.py C3 C5b > gpurun_out/r02aa/sf.log 2>&1
rc=$?
grep -h '^{' gpurun_out/r02aa/sf.log
exit $rc
