set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02j
bash tools/pmc_kernel.sh k_ks_tiled r02j/arb12 python3 tools/ks_bench.py ARB12 --reps 1 > gpurun_out/r02j/arb12.txt 2>&1
rc=$?
cat gpurun_out/r02j/arb12.txt
exit $rc
