#!/bin/bash
# VGPR / spill summary per kernel of one source file: tools/regs.sh blind_rotate_f64 [name filter]
set -eu
cd "$(dirname "$0")/../tfhe-gpu_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-inline-asm -I../include -Icsrc \
  -c csrc/$1.hip -o /tmp/regs_$1.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import sys, re
cur = None
for line in sys.stdin:
    if 'error' in line: print(line, end='')
    m = re.search(r'Function Name: (\S+)', line)
    if m: cur = m.group(1); print(); print(cur[:100], end=' ')
    for k in ('VGPRs:', 'AGPRs:', 'VGPRs Spill:', 'Occupancy \[waves/SIMD\]:'):
        m = re.search(k + r' (\d+)', line)
        if m: print(k.replace('\\\\', ''), m.group(1), end=' ')
print()
" | grep -E "${2:-.}"
