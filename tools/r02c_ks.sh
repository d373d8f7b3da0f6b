set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u -m pytest tests/test_gpu_keyswitch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02c/pytest.log 2>&1 &&
for c in 1 2; do TFHE_KS_CTS=$c timeout -k 10 300 python -u tools/ks_bench.py STD192 STD128Q ARB12 LOGQ23 > gpurun_out/r02c/ks_bench_cts$c.log 2>&1 || exit 1; done
rc=$?
tail -3 gpurun_out/r02c/pytest.log
cat gpurun_out/r02c/ks_bench_cts*.log
exit $rc
