#!/bin/bash
# f64w key-group warm-up by LDS-DMA (TFHE_F64W_PF): N = 2048 parity + WRAP stress, then A/B of
# 0 / 2 / 4 warmed groups on STD192 and STD128Q (device-resident bench), alternating, one box.
# Record only: the switch and the warm-up were removed after this run (profiles/r02bc: slower).
set -u
export TMPDIR=/tmp
D=gpurun_out/r02bc
mkdir -p $D
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "n2048 or wrap or kat or floor_sign" > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python3 -u tools/dbg_wrap.py 6 > $D/wrap.log 2>&1 || { tail -20 $D/wrap.log; exit 1; }
grep -c "\[\]" $D/wrap.log
for rep in 1 2; do
  for pf in 0 2 4; do
    for ps in STD192 STD128Q; do
      TFHE_F64W_PF=$pf timeout -k 10 300 python3 bench.py --params $ps --no-cpu-baseline --steps 3 --warmup 1 > $D/${ps}_pf${pf}_$rep.log 2>&1 || { tail -5 $D/${ps}_pf${pf}_$rep.log; exit 1; }
      echo "$ps pf=$pf rep=$rep $(tail -1 $D/${ps}_pf${pf}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
  done
done
