# sf2 products after every digit's transform (two-digit build for C5b): parity, then C3/C5b A/B
# against gen3sf (TFHE_SF2=0) in the same call.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ad
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "logq or kat or floor_sign" > gpurun_out/r02ad/pytest.log 2>&1 || { tail -5 gpurun_out/r02ad/pytest.log; exit 1; }
tail -1 gpurun_out/r02ad/pytest.log
timeout -k 10 400 python3 tools/bench_configs.py C3 C5b > gpurun_out/r02ad/sf2.log 2>&1 &&
TFHE_SF2=0 timeout -k 10 400 python3 tools/bench_configs.py C3 C5b > gpurun_out/r02ad/gen3sf.log 2>&1
rc=$?
for f in sf2 gen3sf; do grep -h '^{' gpurun_out/r02ad/$f.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$f', d['config'], d['bootstraps_per_s'])"; done
exit $rc
