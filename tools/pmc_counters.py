#!/usr/bin/env python3
"""Per-launch averages of every PMC counter rocprofv3 recorded for one kernel, over one or more -d dirs.
Usage: pmc_counters.py KERNEL_SUBSTRING DIR [DIR ...]   -> one JSON object {counter: mean per launch}"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    kname, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if kname in r.get("Kernel_Name", ""):
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(json.dumps({k: sum(v) / len(v) for k, v in sorted(vals.items())}))


if __name__ == "__main__":
    main()
