"""Model of the 4-wavefront fast kernel's layouts and LDS exchanges (blind_rotate_fast4.hip).
A ciphertext is 256 lanes (4 wavefronts) x 4 registers per polynomial.  A layout names the
index bit (b0..b9 of the natural NTT index) carried by each register bit, lane bit (0..5,
within a wavefront) and wavefront bit.  An exchange A -> B stores every register of A as one
lane-contiguous row (ds_write_addtid_b32) and B gathers with ds_read_b32.  Checks that every
read returns the intended element and that every 32-lane read group hits 32 distinct banks
((a/4) mod 32, MI355X_MICROARCH.md LDS table).  Run: python3 tools/lds_layouts4.py"""
LAY = {  # (register bits, lane bits, wave bits)
    1: ((8, 9), (2, 3, 4, 6, 7, 5), (0, 1)),
    2: ((6, 7), (2, 3, 8, 9, 4, 5), (0, 1)),
    3: ((4, 5), (2, 3, 6, 8, 9, 7), (0, 1)),
    4: ((2, 3), (4, 5, 6, 8, 9, 7), (0, 1)),
    5: ((0, 1), (2, 3, 4, 5, 6, 7), (8, 9)),
}
# exchange (A, B): (row stride of A's register rows, stride of A's wavefront blocks or None if local)
EXCH = {
    (1, 2): (72, None), (2, 3): (80, None), (3, 4): (65, None),
    (2, 1): (68, None), (3, 2): (68, None), (4, 3): (65, None),
    (4, 5): (72, 288), (5, 4): (64, 257),
}


def weight(ex, b):
    """LDS word offset contributed by index bit b in exchange ex (writer-side position)."""
    A, _ = ex
    regs, lanes, waves = LAY[A]
    rs, ws = EXCH[ex]
    if b in regs:
        return rs << regs.index(b)
    if b in lanes:
        return 1 << lanes.index(b)
    if ws is None:
        return 0  # local exchange: the wavefront bits select the wavefront's own region
    return ws << waves.index(b)


def elem(L, wave, lane, r):
    regs, lanes, waves = LAY[L]
    i = 0
    for k, b in enumerate(regs):
        i |= ((r >> k) & 1) << b
    for k, b in enumerate(lanes):
        i |= ((lane >> k) & 1) << b
    for k, b in enumerate(waves):
        i |= ((wave >> k) & 1) << b
    return i


def check(ex):
    A, B = ex
    local = EXCH[ex][1] is None
    # writer memory image
    mem = {}
    for w in range(4):
        for lane in range(64):
            for r in range(4):
                i = elem(A, w, lane, r)
                addr = sum(weight(ex, b) for b in range(10) if (i >> b) & 1)
                key = (w if local else 0, addr)
                assert key not in mem, f"{ex}: address collision"
                mem[key] = i
    extent = max(a for _, a in mem) + 1
    worst = 0
    for w in range(4):
        for r in range(4):
            for g in range(2):
                banks = {}
                for lane in range(32 * g, 32 * g + 32):
                    i = elem(B, w, lane, r)
                    addr = sum(weight(ex, b) for b in range(10) if (i >> b) & 1)
                    assert mem[(w if local else 0, addr)] == i
                    banks.setdefault(addr % 32, set()).add(addr)
                worst = max(worst, max(len(s) for s in banks.values()))
    print(f"exchange L{A}->L{B}: {'local' if local else 'cross'}, extent {extent} words, "
          f"max {worst}-way per 32-lane group")
    assert worst == 1
    return extent


if __name__ == "__main__":
    for ex in EXCH:
        check(ex)
