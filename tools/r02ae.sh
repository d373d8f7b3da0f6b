# Wave-local exact-FP64 kernel (f64w): parity (N = 2048 sets, WRAP, KATs), then STD192 / STD128Q
# device-resident A/B against the slot-layout kernel (TFHE_F64W=0) and the monomial-table switch.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ae
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "n2048 or wrap or kat" > gpurun_out/r02ae/pytest.log 2>&1 || { tail -30 gpurun_out/r02ae/pytest.log; exit 1; }
tail -1 gpurun_out/r02ae/pytest.log
rc=0
for cfg in "TFHE_F64W=1" "TFHE_F64W=0" "TFHE_F64W_MT=1" "TFHE_F64W_MT=0"; do
  for ps in STD192 STD128Q; do
    env $cfg timeout -k 10 300 python3 bench.py --params $ps --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02ae/${ps}_$cfg.log 2>&1 || { rc=1; break 2; }
    echo "$ps $cfg $(tail -1 gpurun_out/r02ae/${ps}_$cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
exit $rc
