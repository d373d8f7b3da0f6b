# fast4 key-stream locality (timing only, results invalid): variant 66 reads rounds 0-7's key
# rows (L2-resident) against the default 60, with one PMC clock pass each.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02al
export TFHE_TIMING_EXPERIMENTS=1
rc=0
for v in 60 66 60 66; do
  TFHE_FAST_VARIANT=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r02al/v$v.log 2>&1 || { rc=1; break; }
  echo "variant $v $(tail -1 gpurun_out/r02al/v$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
done
[ $rc = 0 ] && VARS="60 66" bash tools/pmc_clock.sh
exit $rc
