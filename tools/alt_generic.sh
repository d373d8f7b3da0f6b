#!/bin/bash
# Build a test-library variant with extra defines for blind_rotate_generic.hip (A/B of its compile-time
# knobs, e.g. SFD_KPRE): altlib/TAG/libtfhe_hip_test.so from the tree's other test objects.
#   tools/alt_generic.sh TAG "-DSFD_KPRE=4 ..."      (container; the .so travels to the GPU box)
set -eu
TAG=$1; DEFS=$2
cd "$(dirname "$0")/../tfhe-gpu_amd"
make -s -j8 lib/libtfhe_hip_test.so
mkdir -p ../altlib/$TAG
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-inline-asm -Wno-unused-value -Wno-unused-result -I../include -Icsrc"
$CXX -mllvm -pragma-unroll-threshold=100000 -DTFHE_TEST_PROBES $DEFS -c csrc/blind_rotate_generic.hip \
  -o ../altlib/$TAG/generic.o
OBJS=$(ls build/*.o | grep -v "blind_rotate_generic\|blind_rotate_f64.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -pthread -o ../altlib/$TAG/libtfhe_hip_test.so $OBJS ../altlib/$TAG/generic.o
rm ../altlib/$TAG/generic.o
echo "built altlib/$TAG/libtfhe_hip_test.so ($DEFS)"
