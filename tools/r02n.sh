set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02n
for p in 1 2 4 8; do
  TFHE_HOST_PARTS=$p timeout -k 10 200 python3 tools/bench_configs.py C2host --reps 3 > gpurun_out/r02n/parts$p.log 2>&1 || exit 1
done
for p in 1 2 4 8; do echo "== parts $p"; grep -v amdgpu.ids gpurun_out/r02n/parts$p.log | tail -5; done
