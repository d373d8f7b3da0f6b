# sf2 timing experiments (results invalid): 1 no key stream (round 0's keys), 2 cached monomials,
# 4 inverse twiddles from LDS, 7 all three; plus a PMC pass on the default build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r02z
export TFHE_TIMING_EXPERIMENTS=1
rc=0
for e in 0 1 2 4 7 0; do
  TFHE_SF2_EXP=$e timeout -k 10 300 python3 tools/bench_configs.py C3 --reps 1 > gpurun_out/r02z/c3_e$e.log 2>&1 || { rc=1; break; }
  echo "exp=$e $(grep -o '"bootstraps_per_s": [0-9.]*' gpurun_out/r02z/c3_e$e.log)"
done
[ $rc = 0 ] && timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/r02z/pmc -o run --output-format csv -- python3 tools/bench_configs.py C3 --reps 1 > gpurun_out/r02z/pmc.log 2>&1
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob("gpurun_out/r02z/pmc/**/*counter_collection.csv", recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "blind_rotate" in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, c in list(agg.items())[:2]:
        g = c["GRBM_GUI_ACTIVE"]
        print(d, {k: f"{v:.4g}" for k, v in c.items()}, "valu_busy", round(c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (g / 8), 3))
PY
exit $rc
