set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02p
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r02p/prof -o run --output-format csv -- python3 tools/host_path_bench.py --parts 4 --reps 2 > gpurun_out/r02p/log.txt 2>&1
rc=$?
ls gpurun_out/r02p/prof
exit $rc
