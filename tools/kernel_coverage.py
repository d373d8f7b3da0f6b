#!/usr/bin/env python3
"""Which kernel instances of a library the GPU test suite ran (every shipped kernel
instance appears in a parity test).

    python3 tools/kernel_coverage.py KERNEL_STATS_CSV LIB.so [LIB2.so]

KERNEL_STATS_CSV: rocprofv3 --kernel-trace --stats of `pytest -m gpu tests` (tools/r04_measure.sh suite).
Lists every __global__ instance in the libraries (host stubs, `nm -C`) with its launch count in the run;
exit status 1 if a product-library instance never ran.
"""
import csv
import re
import subprocess
import sys


def instances(lib):
    out = subprocess.run(["nm", "-C", lib], capture_output=True, text=True, check=True).stdout
    names = set()
    for line in out.splitlines():
        m = re.search(r"__device_stub__(.*)$", line)
        if m:
            names.add(norm(m.group(1)))
    return sorted(names)


def norm(name):
    """'void tfhe::(anonymous namespace)::k<...>(args)' -> 'tfhe::(anonymous namespace)::k<...>'"""
    name = re.sub(r"^void ", "", name.strip())
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):  # drop the argument list: the first '(' at template depth 0 after the name
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0 and name[i - 1] not in ":":
            cut = i
            break
    name = name[:cut].strip()
    m = re.search(r"(?:^|::)(k_\w+.*)$", name)  # the kernel's own name (namespaces dropped)
    return m.group(1) if m else name


def main():
    stats, libs = sys.argv[1], sys.argv[2:]
    ran = {}
    for r in csv.DictReader(open(stats)):
        ran[norm(r["Name"])] = ran.get(norm(r["Name"]), 0) + int(r["Calls"])
    missing = 0
    for k, lib in enumerate(libs):
        print(f"== {lib}")
        for inst in instances(lib):
            n = ran.get(inst, 0)
            print(f"{n:8d}  {inst}")
            if n == 0 and k == 0:
                missing += 1
    print(f"product-library instances never launched by the suite: {missing}")
    sys.exit(1 if missing else 0)


if __name__ == "__main__":
    main()
