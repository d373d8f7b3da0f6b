set -u
O=gpurun_out/r06m; mkdir -p $O
for r in 1 2; do
  for L in tfhe-gpu_amd/lib/libtfhe_hip_test.so altlib/kpre4/libtfhe_hip_test.so altlib/kpre0/libtfhe_hip_test.so; do
    n=$(basename $(dirname $(dirname $L)))_$(basename $(dirname $L))
    echo "[$(date +%T)] $L round $r"
    timeout -k 10 200 python3 -u tools/duo_probe.py --ctx ARB12 --lib $L --reps 5 >> $O/arb_probe.log 2>&1 || exit 1
    timeout -k 10 200 python3 -u tools/small_batch.py duo2 --lib $L --reps 5 >> $O/duo2.log 2>&1 || exit 1
  done
done
echo done
