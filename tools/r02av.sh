# WRAP-correction parity failure seen in the r02at full-suite run (STD128Q_OPT, ciphertext 0):
# repeated scenario on the current build and on the build before the N = 2048 register-pressure
# commit (altlib/libtfhe_hip_pre51.so), then the fast4 MAC A/B (tools/r02au.sh).
set -u
export TMPDIR=/tmp
D=gpurun_out/r02av
mkdir -p $D
timeout -k 10 300 python3 -u tools/dbg_wrap.py 6 > $D/wrap_new.log 2>&1 || { cat $D/wrap_new.log; exit 1; }
cat $D/wrap_new.log
TFHE_LIB=$PWD/altlib/libtfhe_hip_pre51.so timeout -k 10 300 python3 -u tools/dbg_wrap.py 6 > $D/wrap_pre51.log 2>&1 || { cat $D/wrap_pre51.log; exit 1; }
cat $D/wrap_pre51.log
bash tools/r02au.sh
