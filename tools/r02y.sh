# Wave-local special-form kernel (sf2, one digit): parity, then C3/C5b A/B against gen3sf (TFHE_SF2=0).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02y
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "logq or kat" > gpurun_out/r02y/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r02y/pytest.log
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python3 tools/bench_configs.py C3 > gpurun_out/r02y/rns.log 2>&1 &&
TFHE_SF2=0 timeout -k 10 400 python3 tools/bench_configs.py C3 > gpurun_out/r02y/gen.log 2>&1
rc=$?
grep -h '^{' gpurun_out/r02y/rns.log gpurun_out/r02y/gen.log
exit $rc
