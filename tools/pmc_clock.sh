#!/bin/bash
# Clock the chip holds and VALU-busy fraction per kernel variant (one PMC pass each, no tracing domains).
# Usage (GPU box, repo root): tools/pmc_clock.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARS:-60 62 70}; do
  TFHE_TIMING_EXPERIMENTS=1 TFHE_FAST_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES -d gpurun_out/clk_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/clk_$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py k_blind_rotate gpurun_out/clk_$v gpurun_out/clk_$v gpurun_out/clk_$v.json gpurun_out/clk_$v > /dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/clk_$v.json')); g=d['grbm_gui_active_per_launch']; t=d['gui_pass_kernel_ns_per_launch']; print('variant $v', 'kernel_ms', round(t/1e6,2), 'clock_GHz', round(g/8/t,3), 'valu_busy', round(d['sq_insts_valu_per_launch']*4/1024/(g/8),3))"
done
