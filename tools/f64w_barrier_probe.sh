# Timing-only probe (round 3): f64w without the barrier before digit 1's pass A (results invalid); the
# probe build lives in the test library (bench.py --test-lib --knob probe=4).
set -u
mkdir -p gpurun_out/r03fp
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --params STD192 --no-cpu-baseline --no-dropin --no-host-array --steps 2 > gpurun_out/r03fp/base_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r03fp/base_$r.log') if l.startswith('{')][-1]); print('base rep $r', d['roofline']['kernel_ms'])" | tee -a gpurun_out/r03fp/summary.txt
  timeout -k 10 200 python3 bench.py --test-lib --knob probe=4 --params STD192 --no-cpu-baseline --no-dropin --no-host-array --steps 2 > gpurun_out/r03fp/nobar_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r03fp/nobar_$r.log') if l.startswith('{')][-1]); print('no-barrier rep $r', d['roofline']['kernel_ms'])" | tee -a gpurun_out/r03fp/summary.txt
done
