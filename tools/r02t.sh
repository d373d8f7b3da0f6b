# Key-stream locality experiments (timing only, results invalid): every round reads round i&7's
# keys (L2-resident) or i&63's, for the FP64 kernel (STD192, STD128Q) and gen3 u64 (C3).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02t
export TFHE_TIMING_EXPERIMENTS=1
rc=0
for e in 0 1 2 0; do
  for ps in STD192 STD128Q; do
    TFHE_F64_EXP=$e timeout -k 10 300 python3 bench.py --params $ps --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r02t/${ps}_e$e.log 2>&1 || { rc=1; break 2; }
    echo "$ps exp=$e $(tail -1 gpurun_out/r02t/${ps}_e$e.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
  TFHE_GEN3_EXP=$e timeout -k 10 300 python3 tools/bench_configs.py C3 --reps 1 > gpurun_out/r02t/C3_e$e.log 2>&1 || { rc=1; break; }
  echo "C3 exp=$e $(grep '^{' gpurun_out/r02t/C3_e$e.log)"
done
exit $rc
