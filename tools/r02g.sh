set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02g
bash tools/pmc_kernel.sh k_ks_tiled r02g/std128 python3 tools/ks_bench.py STD128 --reps 1 > gpurun_out/r02g/std128.txt 2>&1 &&
bash tools/pmc_kernel.sh k_ks_tiled r02g/arb12 python3 tools/ks_bench.py ARB12 --reps 1 > gpurun_out/r02g/arb12.txt 2>&1
rc=$?
cat gpurun_out/r02g/std128.txt gpurun_out/r02g/arb12.txt
exit $rc
