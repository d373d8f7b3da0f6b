"""Model of the fast kernel's LDS exchanges (blind_rotate_fast.hip): layouts L1..L4,
lane-contiguous (ds_write_addtid_b32) stores, per-lane ds_read_b32 loads.  Checks that
every read returns the intended element and counts bank conflicts per 32-lane group
((a/4) mod 32, MI355X_MICROARCH.md LDS table).  Run: python3 tools/lds_layouts.py"""
LAY = {  # index bit carried by register bit k / lane bit k (lane bit 6 = wavefront)
    1: ((7, 8, 9), (4, 5, 1, 2, 3, 0, 6)),
    2: ((4, 5, 6), (1, 2, 3, 7, 8, 0, 9)),
    3: ((1, 2, 3), (4, 5, 6, 7, 8, 0, 9)),
    4: ((0, 1, 2), (4, 5, 6, 7, 8, 3, 9)),
}
PS, WS = 576, 1152          # poly stride, region (reader wavefront) stride, in words
EXCH = {  # (writer, reader): (row bits, row stride)
    (1, 2): ((7, 8, 6), 65), (2, 1): ((4, 5, 9), 72),
    (2, 3): ((4, 5, 6), 65), (3, 4): ((1, 2, 3), 65),
    (4, 3): ((0, 1, 2), 65), (3, 2): ((1, 2, 3), 65),
}


def weight(ex, b):
    A, B = ex
    rowbits, rs = EXCH[ex]
    if b == LAY[B][1][6]:
        return WS
    if b in rowbits:
        return rs << rowbits.index(b)
    k = LAY[A][1].index(b)
    assert k < 6
    return 1 << k


def elem(L, lane, r):
    regs, lanes = LAY[L]
    i = 0
    for k, b in enumerate(regs):
        i |= ((r >> k) & 1) << b
    for k, b in enumerate(lanes):
        i |= ((lane >> k) & 1) << b
    return i


def addr(ex, i):
    return sum(weight(ex, b) for b in range(10) if (i >> b) & 1)


def check():
    worst = 1
    for ex in EXCH:
        A, B = ex
        mem = {}
        for lane in range(128):      # writer: register r of a wavefront = one 64-word row
            for r in range(8):
                i = elem(A, lane, r)
                a = addr(ex, i)
                w = lane >> 6
                # store address must be lane-contiguous: base(w, r) + (lane & 63)
                base = addr(ex, elem(A, lane & 64, r))
                assert a == base + (lane & 63), (ex, lane, r)
                assert a not in mem
                mem[a] = i
                assert a < 2 * WS
        for w in range(2):
            for r in range(8):
                for half in range(2):
                    banks = {}
                    for l in range(32):
                        lane = w * 64 + half * 32 + l
                        i = elem(B, lane, r)
                        a = addr(ex, i)
                        assert mem[a] == i
                        assert a // WS == w      # a wavefront reads only its own region
                        banks.setdefault(a % 32, set()).add(a)
                    worst = max(worst, max(len(v) for v in banks.values()))
        print(f"exchange L{A}->L{B}: reads conflict-free" if worst == 1 else f"L{A}->L{B}: worst {worst}-way")
    return worst


if __name__ == "__main__":
    assert check() == 1
