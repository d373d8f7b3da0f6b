# PMC (VALU instructions, busy, clock) of the round-2 N = 2048 kernels: f64w on STD192 and
# STD128Q (device-resident bench), sf2 on C3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ag
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/r02ag/std192 -o run --output-format csv -- python3 bench.py --params STD192 --no-cpu-baseline --steps 1 --warmup 0 --kernel-reps 1 > gpurun_out/r02ag/std192.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/r02ag/std128q -o run --output-format csv -- python3 bench.py --params STD128Q --no-cpu-baseline --steps 1 --warmup 0 --kernel-reps 1 > gpurun_out/r02ag/std128q.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/r02ag/c3 -o run --output-format csv -- python3 tools/bench_configs.py C3 --reps 1 > gpurun_out/r02ag/c3.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, collections
for tag in ("std192", "std128q", "c3"):
    for f in glob.glob(f"gpurun_out/r02ag/{tag}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        ns = {}
        for r in csv.DictReader(open(f)):
            if "blind_rotate" in r["Kernel_Name"]:
                agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                ns[r["Dispatch_Id"]] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
        for d, c in list(agg.items())[-1:]:
            g = c["GRBM_GUI_ACTIVE"]
            print(tag, f"kernel {ns[d]/1e6:.1f} ms", f"clock {g/8/ns[d]:.2f} GHz", f"VALU/launch {c['SQ_INSTS_VALU']:.3g}",
                  "valu_busy", round(c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (g / 8), 3))
PY
exit $rc
