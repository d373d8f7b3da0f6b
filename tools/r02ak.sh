# Final-tree validation after removing the experiment hooks: full GPU suite, smoke, rocprofv3
# kernel stats over every SURVEY 8(d) configuration, 2-rank gloo rehearsal of bench.py (both
# ranks share the one GPU).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ak
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ak/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02ak/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02ak/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02ak/smoke.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02ak/kt -o run --output-format csv -- python3 tools/bench_configs.py C3 C4 C5a C5b --reps 1 > gpurun_out/r02ak/configs.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline > gpurun_out/r02ak/bench_2rank_gloo.log 2>&1
rc=$?
tail -1 gpurun_out/r02ak/smoke.log
grep -h '^{' gpurun_out/r02ak/configs.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], d['kernel'], d['bootstraps_per_s'])"
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r02ak/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:70], r["Calls"], f'{float(r["AverageNs"])/1e6:.2f} ms', r["Percentage"])
PY
grep -h '^{' gpurun_out/r02ak/bench_2rank_gloo.log | cut -c1-200
exit $rc
