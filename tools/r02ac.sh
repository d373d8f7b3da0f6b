# FP64 kernel monomial tables A/B in one call (TFHE_F64_MT=1 tables, 0 gathers): STD192 and
# STD128Q device-resident, C4 / C5a host-array; parity of the default build first.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ac
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "n2048 or wrap or custom_modulus" > gpurun_out/r02ac/pytest.log 2>&1 || { tail -5 gpurun_out/r02ac/pytest.log; exit 1; }
tail -1 gpurun_out/r02ac/pytest.log
rc=0
for mt in 1 0 1 0; do
  for ps in STD192 STD128Q; do
    TFHE_F64_MT=$mt timeout -k 10 300 python3 bench.py --params $ps --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02ac/${ps}_mt$mt.log 2>&1 || { rc=1; break 2; }
    echo "$ps mt=$mt $(tail -1 gpurun_out/r02ac/${ps}_mt$mt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
exit $rc
