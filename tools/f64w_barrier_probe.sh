set -u
mkdir -p gpurun_out/r03fp
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --params STD192 --no-cpu-baseline --no-dropin --no-host-array --steps 2 > gpurun_out/r03fp/base_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r03fp/base_$r.log') if l.startswith('{')][-1]); print('base rep $r', d['roofline']['kernel_ms'])" | tee -a gpurun_out/r03fp/summary.txt
  TFHE_TIMING_EXPERIMENTS=1 TFHE_F64W_PROBE=4 timeout -k 10 200 python3 bench.py --params STD192 --no-cpu-baseline --no-dropin --no-host-array --steps 2 > gpurun_out/r03fp/nobar_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r03fp/nobar_$r.log') if l.startswith('{')][-1]); print('no-barrier rep $r', d['roofline']['kernel_ms'])" | tee -a gpurun_out/r03fp/summary.txt
done
