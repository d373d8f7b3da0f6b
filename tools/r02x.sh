# gen3sf: PMC pass (VALU instructions, busy, clock) and kernel-trace stats on C3
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02x
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/r02x/pmc -o run --output-format csv -- python3 tools/bench_configs.py C3 --reps 1 > gpurun_out/r02x/pmc.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02x/kt -o run --output-format csv -- python3 tools/bench_configs.py C3 --reps 1 > gpurun_out/r02x/kt.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob("gpurun_out/r02x/pmc/**/*counter_collection.csv", recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "blind_rotate" in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, c in agg.items():
        g = c["GRBM_GUI_ACTIVE"]
        print(d, {k: f"{v:.4g}" for k, v in c.items()}, "valu_busy", round(c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (g / 8), 3))
for f in glob.glob("gpurun_out/r02x/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:60], r["Calls"], r["AverageNs"], r["Percentage"])
PY
exit $rc
