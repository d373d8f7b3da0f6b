set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "host_pipeline or device_then_host or batch_above or gate_batch_sizes or full_batch" > gpurun_out/r02o/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/host_path_bench.py --parts 1,2,4,8 > gpurun_out/r02o/host_path.log 2>&1
rc=$?
tail -3 gpurun_out/r02o/pytest.log
grep -v amdgpu.ids gpurun_out/r02o/host_path.log
exit $rc
