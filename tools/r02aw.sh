# Bisect of the f64w nondeterminism (r02av): variant B = keys by global loads, variant C = slot
# exponents without the opaque per-round copy; the rest of the 51071bb changes kept in each.
set -u
export TMPDIR=/tmp
D=gpurun_out/r02aw
mkdir -p $D
for v in B C; do
  TFHE_LIB=$PWD/altlib/libtfhe_hip_var$v.so timeout -k 10 300 python3 -u tools/dbg_wrap.py 6 > $D/wrap_var$v.log 2>&1 || { cat $D/wrap_var$v.log; exit 1; }
  cat $D/wrap_var$v.log
done
