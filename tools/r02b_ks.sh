set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyswitch.py tests/test_gpu_mul_matrix.py "tests/test_gpu_parity.py::test_device_then_host_calls_without_sync" "tests/test_gpu_parity.py::test_mkm_parity" -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/ks_bench.py > gpurun_out/r02b/ks_bench.log 2>&1
rc=$?
tail -5 gpurun_out/r02b/pytest.log
cat gpurun_out/r02b/ks_bench.log
exit $rc
