set -u
for b in 1536 3072 4608 6144 7680 8192 9216; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 2 --batch $b > gpurun_out/tail_$b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/tail_$b.log') if l.startswith('{')][-1]); print($b, d['roofline']['kernel_ms'], d['value'])"
done
