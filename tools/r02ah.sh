# Last digit's forward outputs kept in LDS (f64w, sf2): parity, then A/B against the previous
# build (altlib/libtfhe_hip_prev.so, TFHE_LIB) in the same call.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ah
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "logq or n2048 or wrap or kat or floor_sign" > gpurun_out/r02ah/pytest.log 2>&1 || { tail -30 gpurun_out/r02ah/pytest.log; exit 1; }
tail -1 gpurun_out/r02ah/pytest.log
rc=0
for lib in new prev new prev; do
  L=""; [ $lib = prev ] && L="TFHE_LIB=$PWD/altlib/libtfhe_hip_prev.so"
  for ps in STD192 STD128Q; do
    env $L timeout -k 10 300 python3 bench.py --params $ps --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02ah/${ps}_$lib.log 2>&1 || { rc=1; break 2; }
    echo "$ps $lib $(tail -1 gpurun_out/r02ah/${ps}_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
  env $L timeout -k 10 400 python3 tools/bench_configs.py C3 C5b > gpurun_out/r02ah/cfg_$lib.log 2>&1 || { rc=1; break; }
  grep -h '^{' gpurun_out/r02ah/cfg_$lib.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config'], '$lib', d['bootstraps_per_s'])"
done
exit $rc
