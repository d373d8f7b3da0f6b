# FP64 kernel: barrier cost (timing only, results invalid: TFHE_F64_EXP=4 drops the transforms'
# barriers) and a PMC pass (VALU instructions, clock) on the default build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02u
export TFHE_TIMING_EXPERIMENTS=1
rc=0
for e in 0 4 0 4; do
  for ps in STD192 STD128Q; do
    TFHE_F64_EXP=$e timeout -k 10 300 python3 bench.py --params $ps --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r02u/${ps}_e$e.log 2>&1 || { rc=1; break 2; }
    echo "$ps exp=$e $(tail -1 gpurun_out/r02u/${ps}_e$e.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
[ $rc = 0 ] && for ps in STD192 STD128Q; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/r02u/pmc_$ps -o run --output-format csv -- python3 bench.py --params $ps --no-cpu-baseline --steps 1 --warmup 0 --kernel-reps 1 > gpurun_out/r02u/pmc_$ps.log 2>&1 || { rc=1; break; }
done
exit $rc
