# Non-fold digit shapes issue digit 0's key rows at the start of each round (no spills): parity
# of the four shapes on the fast path, then F11 / F11t0 host-array throughput and kernel stats.
set -u
export TMPDIR=/tmp
D=gpurun_out/r02ao
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "digit_shapes or std128_opt or reference_kat" \
  > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o f11 --output-format csv -- python3 tools/bench_configs.py F11 F11t0 --reps 3 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
grep '^{' $D/prof.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $D/bench.log 2>&1 || exit 1
tail -1 $D/bench.log | cut -c1-200
