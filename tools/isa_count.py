"""Per-basic-block instruction counts of one kernel in a hipcc --save-temps .s file.
Usage: python3 tools/isa_count.py FILE.s SYMBOL_SUBSTRING
Prints each block's VALU / LDS / VMEM / SALU / scratch counts and the branch that ends
it, so a loop body's per-iteration cost can be read off (used for the blind-rotation
round: outer body + 4 x digit body)."""
import re
import sys
from collections import Counter

path, sym = sys.argv[1], sys.argv[2]
text = open(path).read()
m = re.search(r"^(\S*%s\S*):[^\n]*\n(.*?)^\.Lfunc_end" % re.escape(sym), text, re.S | re.M)
if not m:
    sys.exit("symbol not found")
print(m.group(1))
block, cnt, total = "entry", Counter(), Counter()


def flush(term):
    if sum(cnt.values()):
        print(f"{block:14s} valu {cnt['valu']:5d} lds {cnt['lds']:4d} vmem {cnt['vmem']:3d} "
              f"salu {cnt['salu']:4d} scratch {cnt['scratch']:3d} waitcnt {cnt['wait']:3d}  {term}")


for raw in m.group(2).split("\n"):
    line = raw.split(";")[0].strip()
    if not line or line.startswith("."):
        if line.startswith(".LBB"):
            pass
        else:
            continue
    if re.match(r"^\.LBB\S*:$", line):
        flush("")
        block, cnt = line[:-1], Counter()
        continue
    op = line.split()[0]
    if op.startswith("scratch_") or (op.startswith("buffer_") and "off" in line):
        cnt["scratch"] += 1
    if op.startswith("v_"):
        cnt["valu"] += 1
    elif op.startswith("ds_"):
        cnt["lds"] += 1
    elif op.startswith(("global_", "buffer_", "scratch_")):
        cnt["vmem"] += 1
    elif op == "s_waitcnt":
        cnt["wait"] += 1
    elif op.startswith("s_"):
        cnt["salu"] += 1
    total.update(cnt) if False else None
    if op.startswith("s_cbranch") or op == "s_branch":
        flush(line)
        block, cnt = block + "+", Counter()
flush("end")
