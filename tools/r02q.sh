set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02q
for rep in 1 2; do
TFHE_KS_TILED_MIN=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02q/gather_$rep.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02q/tiled_$rep.log 2>&1 || exit 1
done
for f in gpurun_out/r02q/*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"; done
