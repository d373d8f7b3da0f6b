# gen3 (generic N = 2048, u32 / u64 Shoup) with LDS monomial tables: parity on STD256/STD256Q and
# forced-generic STD192 / logQ paths, then STD256Q / STD256 device-resident A/B against the
# previous build (altlib/libtfhe_hip_prev.so).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02aj
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paramsets.py -x -q --timeout 120 --timeout-method thread -k "generic or paramset or STD256" > gpurun_out/r02aj/pytest.log 2>&1 || { tail -30 gpurun_out/r02aj/pytest.log; exit 1; }
tail -1 gpurun_out/r02aj/pytest.log
rc=0
for lib in new prev; do
  L=""; [ $lib = prev ] && L="TFHE_LIB=$PWD/altlib/libtfhe_hip_prev.so"
  for ps in STD256Q STD256; do
    env $L timeout -k 10 300 python3 bench.py --params $ps --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r02aj/${ps}_$lib.log 2>&1 || { rc=1; break 2; }
    echo "$ps $lib $(tail -1 gpurun_out/r02aj/${ps}_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
exit $rc
