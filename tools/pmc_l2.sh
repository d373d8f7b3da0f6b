#!/bin/bash
# L2 / memory-side split of the blind rotation: one --pmc pass per configuration with
# TCC_HIT_sum, TCC_MISS_sum (L2 hit rate), TCC_EA0_RDREQ_sum (every L2 -> fabric read request; FETCH_SIZE is
# built from it) and TCC_EA0_RDREQ_DRAM_sum (those destined for the memory controllers, i.e. Infinity Cache
# or HBM; the rest go to IO / other dies).  No counter on this stack separates Infinity-Cache hits from HBM
# reads.  Usage (GPU box, repo root): tools/pmc_l2.sh TAG "C2 C3"
set -u
TAG=$1
CFGS=$2
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for CFG in $CFGS; do
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum \
    -d $O/pmcl2_$CFG -o run --output-format csv -- python3 bench.py --config $CFG --no-cpu-baseline --no-host-array \
    --no-dropin --steps 1 --warmup 1 --kernel-reps 1 > $O/pmcl2_$CFG.log 2>&1 || exit $?
  python3 - $O/pmcl2_$CFG $CFG <<'PY' > $O/pmcl2_$CFG.json || exit $?
import collections, csv, glob, json, sys
d, cfg = sys.argv[1:3]
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_blind_rotate" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
out = {"config": cfg, "kernel": "k_blind_rotate*", "launches": max(len(v) for v in agg.values()), "per_launch": m}
h, mi = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
if h is not None and mi:
    out["l2_hit_rate"] = round(h / (h + mi), 4)
if m.get("TCC_EA0_RDREQ_sum"):
    out["dram_share_of_ea_reads"] = round(m.get("TCC_EA0_RDREQ_DRAM_sum", 0) / m["TCC_EA0_RDREQ_sum"], 4)
    out["ea_read_bytes_per_launch_128B"] = m["TCC_EA0_RDREQ_sum"] * 128
print(json.dumps(out))
PY
  cat $O/pmcl2_$CFG.json
done
