set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02k
timeout -k 10 300 python -u -m pytest tests/test_gpu_keyswitch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02k/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/ks_bench.py > gpurun_out/r02k/ks_bench_cts1.log 2>&1 &&
true
rc=$?
tail -3 gpurun_out/r02k/pytest.log
cat gpurun_out/r02k/ks_bench_cts*.log
exit $rc
