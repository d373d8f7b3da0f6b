#!/bin/bash
# Builds altlib/libtfhe_hip_ai{1..4}.so: the tree library with blind_rotate_f64.hip compiled under
# -DTFHE_AI_PROBE=k (the a_i load forms of k_blind_rotate_f64w, see the source).  Container only.
set -eu
cd "$(dirname "$0")/.."
make -s -C tfhe-gpu_amd -j8
mkdir -p altlib/obj
OBJS=$(ls tfhe-gpu_amd/build/*.o | grep -v blind_rotate_f64.o)
for k in ${@:-1 2 3 4}; do
  (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result \
      -Wno-unused-value -Wno-inline-asm -Iinclude -Itfhe-gpu_amd/csrc -DTFHE_AI_PROBE=$k \
      -c tfhe-gpu_amd/csrc/blind_rotate_f64.hip -o altlib/obj/f64_ai$k.o &&
   /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -pthread -o altlib/libtfhe_hip_ai$k.so \
      $OBJS altlib/obj/f64_ai$k.o) &
done
wait
ls -la altlib/*.so
