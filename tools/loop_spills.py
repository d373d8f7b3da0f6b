#!/usr/bin/env python3
"""Scratch (spill) instructions of one kernel in a device .s file, split into inside / outside its
largest loop (the round loop).  Usage: tools/loop_spills.py file.s name-substring"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    names = [m.group(1) for m in re.finditer(r'^(_Z\S+):', s, re.M) if sys.argv[2] in m.group(1)]
    for name in names:
        i = s.index(name + ':')
        j = s.index('.Lfunc_end', i)
        b = s[i:j].split('\n')
        labels = {}
        for k, l in enumerate(b):
            m = re.match(r'(\.LBB\d+_\d+):', l)
            if m:
                labels[m.group(1)] = k
        loops = []
        for k, l in enumerate(b):
            m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
            if m and m.group(1) in labels and labels[m.group(1)] < k:
                loops.append((labels[m.group(1)], k))
        big = max(loops, key=lambda x: x[1] - x[0]) if loops else (0, -1)
        sc = [k for k, l in enumerate(b) if 'scratch_' in l]
        inl = [k for k in sc if big[0] <= k <= big[1]]
        ninstr = sum(1 for l in b[big[0]:big[1] + 1] if l.startswith('\t') and not l.strip().startswith(('.', ';')))
        print(f"{name[:90]}: loop {ninstr} instr, scratch in loop {len(inl)} "
              f"(loads {sum('load' in b[k] for k in inl)}, stores {sum('store' in b[k] for k in inl)}), outside {len(sc) - len(inl)}")


if __name__ == "__main__":
    main()
