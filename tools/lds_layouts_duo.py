#!/usr/bin/env python3
"""Checks the split transforms of the two-workgroup FP64 blind rotation (blind_rotate_f64.hip
f64d_fwd / f64d_inv, k_blind_rotate_f64wduo).

1. Index algebra: member h's forward (stage 0 for half h's outputs, stages 1-2 across waves, then the
   wave-local radix-4 passes (3,4) (5,6) (7,8) (9,10)), run with the kernel's thread -> element and
   twiddle formulas, yields exactly half h of the plain stage-by-stage CT transform at the slots the
   kernel says (lane l of wave w: slots 4u .. 4u+3, u = 64 (w & 3) + l of half h, polynomial w >> 2);
   the inverse (units (10,9), passes (8,7) (6,5) (4,3) wave-local, (2,1) across waves, the hand-off,
   stage 0 for all coefficients) equals the plain GS loop.  Random twiddle tables mod a prime, so
   every index matters.
2. Wave locality: every wave-local pass of wave w touches only its own 256-block (w & 3) of polynomial
   w >> 2's half buffer.
3. LDS banks (MI355X_MICROARCH.md "LDS"): every ds_read_b64 through dswz() touches 32 distinct double
   slots mod 32 per 32-lane group (64 four-byte banks), and every ds_write_b64 16 distinct slots mod 16 per
   16-lane group (32 banks), for every pass, the D / C' exchange (writes of this column's slots, reads of
   the other polynomial's) and the units.
Usage: python3 tools/lds_layouts_duo.py   (run by tests/test_layouts.py)
"""
import random
import sys

N, H, TH, P = 2048, 1024, 512, 1000000007


def dswz(x):
    return x ^ (((x >> 5) & 1) * 10) ^ (((x >> 6) & 1) << 4) ^ (((x >> 4) & 1) * 5)


def ref_fwd(a, psi):
    a = a[:]
    m = 1
    while m < N:
        h = N // (2 * m)
        for i in range(m):
            for j in range(i * 2 * h, i * 2 * h + h):
                v = a[j + h] * psi[m + i] % P
                a[j], a[j + h] = (a[j] + v) % P, (a[j] - v) % P
        m *= 2
    return a


def ref_inv(a, ipsi):
    a = a[:]
    h = 1
    while h < N:
        m = N // (2 * h)
        for i in range(m):
            for j in range(i * 2 * h, i * 2 * h + h):
                x, y = a[j], a[j + h]
                a[j], a[j + h] = (x + y) % P, (x - y) * ipsi[m + i] % P
        h *= 2
    return a


def ct(v, i, j, w):
    t = v[j] * w % P
    v[i], v[j] = (v[i] + t) % P, (v[i] - t) % P


def gs(v, i, j, w):
    x, y = v[i], v[j]
    v[i], v[j] = (x + y) % P, (x - y) * w % P


class Lds:
    """one member's half buffer [2][H] (swizzled within each 256-block) with an access trace"""

    def __init__(self):
        self.m = [None] * (2 * H)
        self.trace = []   # reads: (pass name, instruction index), thread, address
        self.wtrace = []  # writes

    def addr(self, poly, x):
        return poly * H + (x & ~255) + dswz(x & 255)

    def rd(self, tag, t, poly, x):
        a = self.addr(poly, x)
        self.trace.append((tag, t, a))
        return self.m[a]

    def wr(self, tag, t, poly, x, v):
        a = self.addr(poly, x)
        self.wtrace.append((tag, t, a))
        self.m[a] = v


def fwd_member(polys, h, psi, lds, wl):
    """polys: two full polynomials; returns d[t] = 4 values of the lane's slots (f64d_fwd)"""
    for t in range(TH):  # pass A (across waves)
        tau, pp = t & 255, t >> 8
        v = [polys[pp][tau + 256 * k] for k in range(8)]
        o = [0] * 4
        for k in range(4):
            x = v[k + 4] * psi[1] % P
            o[k] = (v[k] - x) % P if h else (v[k] + x) % P
        ct(o, 0, 2, psi[2 + h]), ct(o, 1, 3, psi[2 + h])
        ct(o, 0, 1, psi[4 + 2 * h]), ct(o, 2, 3, psi[5 + 2 * h])
        for k in range(4):
            lds.wr(("fA", k), t, pp, 256 * k + tau, o[k])
    d = {}
    for name, ys, tw in [
            ("f34", lambda l: [l + 64 * k for k in range(4)],
             lambda B, l: [(0, 2, 8 + B), (1, 3, 8 + B), (0, 1, 16 + 2 * B), (2, 3, 17 + 2 * B)]),
            ("f56", lambda l: [64 * (l >> 4) + (l & 15) + 16 * k for k in range(4)],
             lambda B, l: [(0, 2, 32 + 4 * B + (l >> 4)), (1, 3, 32 + 4 * B + (l >> 4)),
                           (0, 1, 64 + 8 * B + 2 * (l >> 4)), (2, 3, 65 + 8 * B + 2 * (l >> 4))]),
            ("f78", lambda l: [16 * (l >> 2) + (l & 3) + 4 * k for k in range(4)],
             lambda B, l: [(0, 2, 128 + 16 * B + (l >> 2)), (1, 3, 128 + 16 * B + (l >> 2)),
                           (0, 1, 256 + 32 * B + 2 * (l >> 2)), (2, 3, 257 + 32 * B + 2 * (l >> 2))]),
            ("f910", lambda l: [4 * l + k for k in range(4)],
             lambda B, l: [(0, 2, 512 + 64 * B + l), (1, 3, 512 + 64 * B + l),
                           (0, 1, 1024 + 128 * B + 2 * l), (2, 3, 1025 + 128 * B + 2 * l)])]:
        for t in range(TH):
            w, l = t >> 6, t & 63
            B, poly, blk = 4 * h + (w & 3), w >> 2, w & 3
            xs = [256 * blk + y for y in ys(l)]
            wl.append((name, w, [(poly, x) for x in xs]))
            x4 = [lds.rd((name, k), t, poly, x) for k, x in enumerate(xs)]
            for (i, j, e) in tw(B, l):
                ct(x4, i, j, psi[e])
            if name == "f910":
                d[t] = x4
            else:
                for k, x in enumerate(xs):
                    lds.wr((name, 4 + k), t, poly, x, x4[k])
    return d


def inv_member(s, h, ipsi, lds, wl):
    """s[t] = the lane's 4 slot values of column w >> 2 -> o[t] = 4 values tau + 256k' of half h (f64d_inv)"""
    for name, ys, tw in [
            ("i109", lambda l: [4 * l + k for k in range(4)],
             lambda B, l: [(0, 1, 1024 + 128 * B + 2 * l), (2, 3, 1025 + 128 * B + 2 * l),
                           (0, 2, 512 + 64 * B + l), (1, 3, 512 + 64 * B + l)]),
            ("i87", lambda l: [16 * (l >> 2) + (l & 3) + 4 * k for k in range(4)],
             lambda B, l: [(0, 1, 256 + 32 * B + 2 * (l >> 2)), (2, 3, 257 + 32 * B + 2 * (l >> 2)),
                           (0, 2, 128 + 16 * B + (l >> 2)), (1, 3, 128 + 16 * B + (l >> 2))]),
            ("i65", lambda l: [64 * (l >> 4) + (l & 15) + 16 * k for k in range(4)],
             lambda B, l: [(0, 1, 64 + 8 * B + 2 * (l >> 4)), (2, 3, 65 + 8 * B + 2 * (l >> 4)),
                           (0, 2, 32 + 4 * B + (l >> 4)), (1, 3, 32 + 4 * B + (l >> 4))]),
            ("i43", lambda l: [l + 64 * k for k in range(4)],
             lambda B, l: [(0, 1, 16 + 2 * B), (2, 3, 17 + 2 * B), (0, 2, 8 + B), (1, 3, 8 + B)])]:
        for t in range(TH):
            w, l = t >> 6, t & 63
            B, poly, blk = 4 * h + (w & 3), w >> 2, w & 3
            xs = [256 * blk + y for y in ys(l)]
            wl.append((name, w, [(poly, x) for x in xs]))
            x4 = s[t][:] if name == "i109" else [lds.rd((name, k), t, poly, x) for k, x in enumerate(xs)]
            for (i, j, e) in tw(B, l):
                gs(x4, i, j, ipsi[e])
            for k, x in enumerate(xs):
                lds.wr((name, 4 + k), t, poly, x, x4[k])
    o = {}
    for t in range(TH):  # stages 2, 1 across waves
        tau, pp = t & 255, t >> 8
        v = [lds.rd(("iA", k), t, pp, 256 * k + tau) for k in range(4)]
        gs(v, 0, 1, ipsi[4 + 2 * h]), gs(v, 2, 3, ipsi[5 + 2 * h])
        gs(v, 0, 2, ipsi[2 + h]), gs(v, 1, 3, ipsi[2 + h])
        o[t] = v
    return o


def banks(trace, group):
    """worst number of distinct-address lanes on one bank within a lane group of `group` lanes: reads
    group 32 (double slots mod 32), writes group 16 (slots mod 16)"""
    by = {}
    for tag, t, a in trace:
        by.setdefault(tag, {}).setdefault(t, []).append(a)
    worst = 1
    for tag, per in by.items():
        n = len(next(iter(per.values())))
        for i in range(n):
            for g in range(TH // group):
                slots = [per[t][i] % group for t in range(group * g, group * g + group) if t in per]
                if slots:
                    worst = max(worst, max(slots.count(x) for x in set(slots)))
    return worst


def main():
    rnd = random.Random(5)
    psi = [rnd.randrange(P) for _ in range(N)]
    ipsi = [rnd.randrange(P) for _ in range(N)]
    polys = [[rnd.randrange(P) for _ in range(N)] for _ in range(2)]
    want = [ref_fwd(p, psi) for p in polys]
    ok = True
    S_full = [[rnd.randrange(P) for _ in range(N)] for _ in range(2)]
    inv_want = [ref_inv(S, ipsi) for S in S_full]
    halves = {}
    for h in range(2):
        lds, wl = Lds(), []
        d = fwd_member(polys, h, psi, lds, wl)
        for t in range(TH):
            w, l = t >> 6, t & 63
            u = 256 * h + 64 * (w & 3) + l
            if d[t] != [want[w >> 2][4 * u + k] for k in range(4)]:
                print(f"VIOLATION: forward member {h} thread {t} slots differ")
                ok = False
                break
        # the D / C' exchange: each lane writes its column's 4 slots, then reads the other polynomial's
        for t in range(TH):
            w, l = t >> 6, t & 63
            for k in range(4):
                lds.wtrace.append((("xw", k), t, lds.addr(w >> 2, 256 * (w & 3) + 4 * l + k)))
                lds.rd(("prod", k), t, 1 - (w >> 2), 256 * (w & 3) + 4 * l + k)
        s = {}
        for t in range(TH):
            w, l = t >> 6, t & 63
            u = 256 * h + 64 * (w & 3) + l
            s[t] = [S_full[w >> 2][4 * u + k] for k in range(4)]
        halves[h] = inv_member(s, h, ipsi, lds, wl)
        for name, w, xs in wl:
            if any(p != w >> 2 or not (256 * (w & 3) <= x < 256 * (w & 3) + 256) for p, x in xs):
                print(f"VIOLATION: {name} of wave {w} leaves its block")
                ok = False
        wr_, ww_ = banks(lds.trace, 32), banks(lds.wtrace, 16)
        print(f"member {h}: worst b64 bank multiplicity: reads per 32-lane group {wr_}, writes per 16-lane group {ww_}")
        ok &= wr_ == 1 and ww_ == 1
    # hand-off + stage 0 (both members compute every coefficient)
    for t in range(TH):
        tau, pp = t & 255, t >> 8
        for k in range(4):
            lo, hi = halves[0][t][k], halves[1][t][k]
            a0, a1 = (lo + hi) % P, (lo - hi) * ipsi[1] % P
            if a0 != inv_want[pp][tau + 256 * k] or a1 != inv_want[pp][tau + 1024 + 256 * k]:
                print(f"VIOLATION: inverse thread {t} element {k}")
                ok = False
    assert sorted(dswz(x) for x in range(256)) == list(range(256))
    print("index algebra: split forward / inverse equal the stage loops" if ok else "FAILED")
    print("OK" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
