# fast4 MAC without the re-associated 64-bit adds (24 VALU per wave-round fewer): parity of every
# fast4 build and digit shape, then the headline bench against the previous build (TFHE_LIB),
# same box, alternating.
set -u
export TMPDIR=/tmp
D=gpurun_out/r02au
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernel_variants.py tests/test_gpu_parity.py \
  -k "variant or reference_kat or eval_acc or gate_parity or n1024_digit_shapes or full_batch or std128_opt" \
  > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/new_$r.log 2>&1 || { cat $D/new_$r.log; exit 1; }
  TFHE_LIB=$PWD/altlib/libtfhe_hip_prev.so timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/prev_$r.log 2>&1 || { cat $D/prev_$r.log; exit 1; }
  for f in new_$r prev_$r; do
    echo "$f $(grep '^{' $D/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
