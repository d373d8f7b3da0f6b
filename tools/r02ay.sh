# Fix of the f64w / sf2 intermittent results (a_i mod amod by division again, profiles/r02ax)
# + the fast4 MAC change: WRAP and N = 2048 repeats, full GPU suite, smoke, headline bench +
# rocprofv3 kernel stats, the other configurations.
set -u
export TMPDIR=/tmp
D=gpurun_out/r02ay
mkdir -p $D
timeout -k 10 300 python3 -u tools/dbg_wrap.py 8 > $D/wrap.log 2>&1 || { cat $D/wrap.log; exit 1; }
grep -c "\[(" $D/wrap.log; grep "random a" $D/wrap.log
timeout -k 10 300 python3 -u tools/dbg_ct0.py 4 STD192 arb12 logq23 STD128Q > $D/ct0.log 2>&1 || { cat $D/ct0.log; exit 1; }
grep "reps with" $D/ct0.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { cat $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python3 bench.py > $D/bench.log 2>&1 || { cat $D/bench.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
timeout -k 10 600 python3 tools/bench_configs.py C2host C3 C4 C5a C5b --reps 2 > $D/configs.log 2>&1 || { cat $D/configs.log; exit 1; }
grep -h '^{' $D/bench.log | cut -c1-300
grep -h '^{' $D/configs.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], d['kernel'], d['bootstraps_per_s'])"
