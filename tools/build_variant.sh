#!/bin/bash
# Builds an experiment variant of the product library: blind_rotate_generic.hip, blind_rotate_f64.hip and ks_tiled.hip
# recompiled with extra -D flags, linked with the other objects of tfhe-gpu_amd/build/ (run `make` first).
#   tools/build_variant.sh NAME "-DSF2_MONO_ROWS=0 -DF64W_MONO_ROWS=0"  -> altlib/libtfhe_hip_NAME.so
# (altlib/ is git-ignored and travels to the GPU box; bench.py / tools/ab_lib.sh select it by TFHE_LIB)
set -e
NAME=$1; DEFS=$2
cd "$(dirname "$0")/../tfhe-gpu_amd"
O=/tmp/tfhe_variant_$NAME
mkdir -p $O ../altlib
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result -Wno-unused-value -Wno-inline-asm -I../include -Icsrc"
/opt/rocm/bin/hipcc $F -mllvm -pragma-unroll-threshold=100000 $DEFS -c csrc/blind_rotate_generic.hip -o $O/blind_rotate_generic.o &
/opt/rocm/bin/hipcc $F $DEFS -c csrc/blind_rotate_f64.hip -o $O/blind_rotate_f64.o &
/opt/rocm/bin/hipcc $F $DEFS -c csrc/ks_tiled.hip -o $O/ks_tiled.o &
wait
OBJS=$(ls build/*.o | grep -v -e blind_rotate_generic.o -e blind_rotate_f64.o -e ks_tiled.o -e _probes.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -pthread -o ../altlib/libtfhe_hip_$NAME.so $OBJS $O/blind_rotate_generic.o $O/blind_rotate_f64.o $O/ks_tiled.o
echo "altlib/libtfhe_hip_$NAME.so"
