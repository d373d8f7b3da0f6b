# Special-form u64 kernel (gen3sf): parity on the logQ contexts, then C3/C5b throughput A/B
# against the Shoup gen3 kernel (TFHE_SF=0) in the same call.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02w
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "logq or kat or floor_sign" > gpurun_out/r02w/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r02w/pytest.log
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python3 tools/bench_configs.py C3 C5b > gpurun_out/r02w/rns.log 2>&1 &&
TFHE_SF=0 timeout -k 10 400 python3 tools/bench_configs.py C3 C5b > gpurun_out/r02w/gen.log 2>&1
rc=$?
grep -h '^{' gpurun_out/r02w/rns.log gpurun_out/r02w/gen.log
exit $rc
