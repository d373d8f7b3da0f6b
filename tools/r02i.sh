set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02i
for c in STD128 ARB12; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02i/$c -o run --output-format csv -- python3 tools/ks_bench.py $c > gpurun_out/r02i/$c.log 2>&1 || exit 1
done
for c in STD128 ARB12; do tail -1 gpurun_out/r02i/$c.log; cut -d, -f1-4 gpurun_out/r02i/$c/run_kernel_stats.csv | cut -c1-150; done
