set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02m
bash tools/pmc_kernel.sh k_blind_rotate r02m/c4 python3 bench.py --params STD192 --no-cpu-baseline --steps 1 --warmup 0 --kernel-reps 1 > gpurun_out/r02m/c4.txt 2>&1
rc=$?
cat gpurun_out/r02m/c4.txt
exit $rc
