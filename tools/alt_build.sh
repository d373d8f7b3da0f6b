#!/bin/bash
# Build a test-library variant with extra defines for ONE source file (A/B of its compile-time knobs):
#   tools/alt_build.sh SRC TAG "-DNAME=VALUE ..."   ->   altlib/TAG/libtfhe_hip_test.so
# SRC: blind_rotate_generic | ks_tiled | ... (csrc/SRC.hip); the other objects are the tree's test-library ones.
set -eu
SRC=$1; TAG=$2; DEFS=$3
cd "$(dirname "$0")/../tfhe-gpu_amd"
make -s -j8 lib/libtfhe_hip_test.so
mkdir -p ../altlib/$TAG
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-inline-asm -Wno-unused-value -Wno-unused-result -I../include -Icsrc"
EXTRA="-DTFHE_TEST_PROBES"
[ "$SRC" = blind_rotate_generic ] && EXTRA="$EXTRA -mllvm -pragma-unroll-threshold=100000"
$CXX $EXTRA $DEFS -c csrc/$SRC.hip -o ../altlib/$TAG/alt.o
# the test library's objects, with SRC's replaced (the probe builds of the generic / f64 files are the test ones)
OBJS=""
for o in build/*.o; do
  b=$(basename $o .o)
  case $b in
    blind_rotate_generic|blind_rotate_f64) continue ;;               # product-only objects
    ${SRC}|${SRC}_probes) continue ;;                                 # replaced
  esac
  OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -pthread -o ../altlib/$TAG/libtfhe_hip_test.so $OBJS ../altlib/$TAG/alt.o
rm ../altlib/$TAG/alt.o
echo "built altlib/$TAG/libtfhe_hip_test.so ($SRC: $DEFS)"
