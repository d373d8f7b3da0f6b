# Generalised four-wavefront kernel (logQ = 11 and STD128_AP digit shapes): parity against the
# oracle on the fast and generic paths, the C++ time-estimate example, and the C2 bench line
# (STD128 must be unchanged).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02am
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "digit_shapes or std128_opt or reference_kat" tests/test_gpu_example.py \
  > gpurun_out/r02am/pytest.log 2>&1 || { tail -30 gpurun_out/r02am/pytest.log; exit 1; }
tail -3 gpurun_out/r02am/pytest.log
timeout -k 10 300 ./examples/time_estimate 16384 > gpurun_out/r02am/time_estimate.log 2>&1 || exit 1
cat gpurun_out/r02am/time_estimate.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02am/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r02am/bench.log
