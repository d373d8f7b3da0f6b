# logQ = 11 EvalFloor (F11: thr 1, F11t0: thr 0) on the generalised four-wavefront kernel and on
# generic v2 (TFHE_FORCE_GENERIC=1), host-array API; then rocprofv3 kernel statistics of F11.
set -u
export TMPDIR=/tmp
D=gpurun_out/r02an
mkdir -p $D
timeout -k 10 300 python3 tools/bench_configs.py F11 F11t0 --reps 3 > $D/fast.log 2>&1 || { cat $D/fast.log; exit 1; }
cat $D/fast.log
TFHE_FORCE_GENERIC=1 timeout -k 10 300 python3 tools/bench_configs.py F11 F11t0 --reps 3 > $D/generic.log 2>&1 || { cat $D/generic.log; exit 1; }
cat $D/generic.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o f11 --output-format csv -- python3 tools/bench_configs.py F11 F11t0 --reps 3 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -3
