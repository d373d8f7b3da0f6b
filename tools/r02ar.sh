# Register pressure in the N = 2048 kernels (sf2 and f64w): pass-A twiddles by scalar loads, key
# and inverse-twiddle loads through buffer resources (32-bit lane offsets), a mod amod as a mask,
# slot exponents recomputed, early inverse units for sf2's two digits.  Parity of the N = 2048
# paths, then C3 / C5b / C4 / C5a host-array throughput against the previous build (TFHE_LIB,
# same box, alternating).
set -u
export TMPDIR=/tmp
D=gpurun_out/r02ar
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "logq or reference_kat or floor_sign_decomp or n2048 or wrap_correction" \
  > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for r in 1 2; do
  timeout -k 10 400 python3 tools/bench_configs.py C3 C5b C4 C5a --reps 2 > $D/new_$r.log 2>&1 || { cat $D/new_$r.log; exit 1; }
  TFHE_LIB=$PWD/altlib/libtfhe_hip_prev.so timeout -k 10 400 python3 tools/bench_configs.py C3 C5b C4 C5a --reps 2 > $D/prev_$r.log 2>&1 || { cat $D/prev_$r.log; exit 1; }
  for f in new_$r prev_$r; do
    echo "$f $(grep '^{' $D/$f.log | python3 -c 'import json,sys; print([(d["config"], d["kernel"], d["bootstraps_per_s"]) for d in map(json.loads, sys.stdin)])')"
  done
done
