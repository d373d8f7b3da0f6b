# Bisect of the f64w nondeterminism (r02av, r02aw): D = a mod amod by %, E = no key-round mask, F = both
set -u
export TMPDIR=/tmp
D=gpurun_out/r02ax
mkdir -p $D
for v in D E F; do
  TFHE_LIB=$PWD/altlib/libtfhe_hip_var$v.so timeout -k 10 300 python3 -u tools/dbg_wrap.py 6 > $D/wrap_var$v.log 2>&1 || { cat $D/wrap_var$v.log; exit 1; }
  cat $D/wrap_var$v.log
done
