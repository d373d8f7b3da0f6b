# f64w key-stream locality (timing only, results invalid): rounds read the key rows of round
# i & 7 (L2-resident) against the real stream, STD192 and STD128Q, same box.
set -u
export TMPDIR=/tmp
D=gpurun_out/r02aq
mkdir -p $D
for P in STD192 STD128Q; do
  for m in 0 8 0 8; do
    if [ $m = 0 ]; then
      timeout -k 10 300 python3 bench.py --params $P --no-cpu-baseline --steps 3 --warmup 1 > $D/${P}_real.log 2>&1 || exit 1
      f=$D/${P}_real.log
    else
      TFHE_TIMING_EXPERIMENTS=1 TFHE_F64_KEYROUNDS=$m timeout -k 10 300 python3 bench.py --params $P --no-cpu-baseline --steps 3 --warmup 1 > $D/${P}_k$m.log 2>&1 || exit 1
      f=$D/${P}_k$m.log
    fi
    echo "$P keyrounds=$m $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
