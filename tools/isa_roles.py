"""Where a kernel's round loop spends its VALU instructions, by source line.

Compiles one translation unit with -gline-tables-only (device code only, the build's flags), takes
the largest basic block of KERNEL (the round loop body of the blind rotations; for loops split into
several blocks pass --blocks N to sum the N largest) and attributes every VALU instruction to the
source line of its last `.loc`.  Lines are grouped into roles by the function or statement they
belong to (ROLES below, matched on the source text); the rest is listed by line.

Usage: python3 tools/isa_roles.py SRC.hip KERNEL_SUBSTRING [--blocks N] [--extra "-mllvm ..."]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.environ.get("ISA_ROLES_CSRC", os.path.join(ROOT, "tfhe-gpu_amd", "csrc"))

# role: (file basename, substrings of the source line)
# products: every line of these device_math.hpp functions (found by their definition lines)
PRODUCT_FUNCS = [("modular product (sf_mul)", "uint64_t sf_mul("), ("modular product (fmodmul)", "double fmodmul_f64(")]
ROLES = [
    ("butterfly sums / offsets", "", ["K.Q3 - v", "K.Q2 - v", "x = x + v", "K.Q10 - y", "K.Q9 - y", "s = x + y"]),
    ("folds / reductions", "", ["sf_fold", "(x & ((1ull << SF_K)", "fred(", "csub"]),
    ("digit decomposition", "", ["Qhalf", ">> shift", "<< sh) >> sh", "Khi", "Klo", "__builtin_floor", "Bginv"]),
    ("accumulator update", "", ["acc[p][k] =", "x >= Q ? x - Q"]),
    ("products' sums", "", ["A[kk][s] =", "A[kk][q] =", "S[j][s] =", "S[j][q] ="]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernel")
    ap.add_argument("--blocks", type=int, default=1)
    ap.add_argument("--extra", default="")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               "-gline-tables-only", "--cuda-device-only", "-S", "-Wno-unused-value", "-I", CSRC,
               "-I", os.path.join(ROOT, "include"), a.src, "-o", out] + a.extra.split()
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
        s = open(out).read()
    files, fullpath = {}, {}
    for mf in re.finditer(r'\.file\s+(\d+)\s+("([^"]*)"\s+)?"([^"]+)"', s):
        base = os.path.basename(mf.group(4))
        files[mf.group(1)] = base
        fullpath[base] = os.path.join(mf.group(3) or "", mf.group(4))
    m = re.search(r"^(\S*%s\S*):[^\n]*\n(.*?)^\.Lfunc_end" % re.escape(a.kernel), s, re.S | re.M)
    if not m:
        sys.exit("kernel not found")
    blocks, cur, loc = [], [], None
    for raw in m.group(2).split("\n"):
        t = raw.strip()
        if re.match(r"^\.LBB\S*:$", t):
            blocks.append(cur)
            cur = []
            continue
        mm = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if mm:
            loc = (files.get(mm.group(1), mm.group(1)), int(mm.group(2)))
            continue
        if t.startswith("v_"):
            cur.append(loc)
    blocks.append(cur)
    chosen = sorted(blocks, key=len, reverse=True)[: a.blocks]
    cnt = Counter(x for b in chosen for x in b)
    total = sum(cnt.values())
    srcs = {}

    def text(f, ln):
        if f not in srcs:
            path = os.path.join(CSRC, f)
            if not os.path.exists(path):
                path = fullpath.get(f, "")
            srcs[f] = open(path).read().split("\n") if path and os.path.exists(path) else []
        return srcs[f][ln - 1].strip() if 0 < ln <= len(srcs[f]) else ""

    def enclosing(f, ln):
        """name of the header function a line belongs to (the FP64 intrinsics of __clang_hip_math.h)"""
        text(f, ln)
        for k in range(ln - 1, max(ln - 12, 0), -1):
            mm = re.search(r"\b(__\w+)\(", srcs[f][k - 1]) if k - 1 < len(srcs[f]) else None
            if mm:
                return mm.group(1)
        return "?"

    ranges = []
    text("device_math.hpp", 1)
    dm = srcs["device_math.hpp"]
    for name, sig in PRODUCT_FUNCS:
        for i, line in enumerate(dm):
            if sig in line:
                j = i
                while j < len(dm) and dm[j].rstrip() != "}":
                    j += 1
                ranges.append((name, i + 1, j + 1))
    roles, rest = Counter(), Counter()
    for (f, ln), v in cnt.items():
        t = text(f, ln)
        hit = [name for name, lo, hi in ranges if f == "device_math.hpp" and lo <= ln <= hi]
        if hit:
            roles[hit[0]] += v
            continue
        if f.startswith("__clang"):  # FP64 intrinsics: products and sums cannot be told apart here
            roles[f"FP64 intrinsic {enclosing(f, ln)} (products and sums)"] += v
            continue
        for name, fname, keys in ROLES:
            if (not fname or fname == f) and any(k in t for k in keys):
                roles[name] += v
                break
        else:
            rest[(f, ln)] += v
    print(f"{m.group(1)}\nVALU in the {a.blocks} largest block(s): {total}")
    for name, v in roles.most_common():
        print(f"  {v:6d}  {100 * v / total:5.1f} %  {name}")
    other = sum(rest.values())
    print(f"  {other:6d}  {100 * other / total:5.1f} %  other lines; the largest:")
    for (f, ln), v in rest.most_common(a.top):
        print(f"      {v:5d}  {f}:{ln}  {text(f, ln)[:90]}")


if __name__ == "__main__":
    main()
