#!/bin/bash
# Same-box memory-side A/B of two library builds on one configuration's blind rotation (verdict r5 item 2:
# C3's FETCH_SIZE per launch rose 70.3 -> 94.5 M KiB between the round-4 and round-5 records).  Per build and
# rep: one FETCH_SIZE pass, one TCC_HIT/TCC_MISS/TCC_EA0_RDREQ pass (one counter group per rocprofv3 run, no
# tracing domains) and one event-timed bench line; builds alternate.  Run on the GPU box from the repo root:
#   tools/fetch_ab.sh TAG C3 "LIB_A LIB_B" [reps]
set -u
TAG=$1; CFG=$2; LIBS=$3; R=${4:-2}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
Q="--config $CFG --no-cpu-baseline --no-host-array --no-dropin --steps 1 --warmup 1 --kernel-reps 1"
for r in $(seq 1 $R); do
  i=0
  for L in $LIBS; do
    i=$((i + 1))
    echo "[$(date +%T)] lib$i rep $r ($L)"
    TFHE_ABI_PREV=1 TFHE_LIB=$L timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/f_${i}_$r -o run --output-format csv -- python3 bench.py $Q > $O/f_${i}_$r.log 2>&1 || { echo "rc=$?"; exit 1; }
    TFHE_ABI_PREV=1 TFHE_LIB=$L timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $O/h_${i}_$r -o run --output-format csv -- python3 bench.py $Q > $O/h_${i}_$r.log 2>&1 || { echo "rc=$?"; exit 1; }
    TFHE_ABI_PREV=1 TFHE_LIB=$L timeout -k 10 300 python3 bench.py --config $CFG --no-cpu-baseline --no-host-array --no-dropin --steps 2 --warmup 1 > $O/b_${i}_$r.log 2>&1 || { echo "rc=$?"; exit 1; }
  done
done
python3 - $O "$LIBS" $R <<'PY'
import collections, csv, glob, json, sys
o, libs, R = sys.argv[1], sys.argv[2].split(), int(sys.argv[3])
res = []
for i, L in enumerate(libs, 1):
    for r in range(1, R + 1):
        agg = collections.defaultdict(list)
        for pre in ("f", "h"):
            for f in glob.glob(f"{o}/{pre}_{i}_{r}/**/*counter_collection.csv", recursive=True):
                for row in csv.DictReader(open(f)):
                    if "k_blind_rotate" in row["Kernel_Name"]:
                        agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
        m = {k: sum(v) / len(v) for k, v in agg.items()}
        line = json.loads(open(f"{o}/b_{i}_{r}.log").read().strip().splitlines()[-1])
        h, mi = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
        res.append({"lib": L, "rep": r, "fetch_kib": m.get("FETCH_SIZE"), "l2_hit": round(h / (h + mi), 4) if h + mi else None,
                    "tcc_miss": mi, "ea_rdreq": m.get("TCC_EA0_RDREQ_sum"), "kernel_ms": line["roofline"]["kernel_ms"],
                    "value": line["value"], "parity_ok": line["parity_ok"]})
        print(json.dumps(res[-1]))
json.dump(res, open(f"{o}/fetch_ab.json", "w"), indent=1)
PY
