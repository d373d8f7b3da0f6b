# Round-2 final-tree profile (tools/gpu_profile.sh recipe): bench, rocprofv3 kernel trace + stats
# of the same command, PMC passes (FETCH/WRITE, instruction mix, VALU busy + clock) -> the
# round-2 PMC summary bench.py reads; then every configuration.
set -u
export TMPDIR=/tmp
bash tools/gpu_profile.sh r02 > gpurun_out/gp_r02.log 2>&1
rc=$?
tail -3 gpurun_out/gp_r02.log
[ $rc = 0 ] || exit $rc
timeout -k 10 700 python3 tools/bench_configs.py C2host C3 C4 C5a C5b > gpurun_out/configs_r02.log 2>&1
rc=$?
grep -h '^{' gpurun_out/configs_r02.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], d['kernel'], d['bootstraps_per_s'])"
exit $rc
