#!/usr/bin/env python3
"""Checks the wave-local N = 2048 transform schedule of sf2 (blind_rotate_generic.hip) and f64w
(blind_rotate_f64.hip).

Thread t of the 512 (wave w = t >> 6, lane l = t & 63):
  pass A    polynomial t >> 8, elements tau + 256k (tau = t & 255)          -- the cross exchange
  pass B    polynomial l >> 5, elements 256w + (l & 31) + 32k
  pass C    polynomial l >> 5, elements 32b + o + 4k, b = 8w + ((l >> 2) & 7), o = l & 3
  units     slots 4u .. 4u+3, u = 64w + l, of BOTH polynomials (left in registers)
and the inverse in the mirrored order.  Checked:
1. index algebra: the passes with the kernels' element and twiddle formulas equal the plain
   CT / GS stage loops on both polynomials (random twiddles mod a prime);
2. wave-locality: every element wave w touches in passes B, C and the units (forward and
   inverse) lies in block w (elements 256w .. 256w+255) of either polynomial -- so those
   passes need no workgroup barrier;
3. LDS banks: every 64-bit access of a half-wave (gfx950 serves b64 per half-wave, 64 banks of
   4 bytes) through the XOR swizzle touches 32 distinct bank pairs.
Usage: python3 tools/lds_layouts_wl.py
"""
import random
import sys

import lds_layouts_f64 as base

N, P = base.N, base.P
swz = base.swz


def fwd_passes(a, psi, trace):
    """a: [2][N]; trace[pass][t] = list of (poly, element) in access order"""
    buf = [row[:] for row in a]
    for pas in range(4):
        per = {}
        for t in range(512):
            w, l = t >> 6, t & 63
            acc = []
            if pas == 0:
                p, tau = t >> 8, t & 255
                base.r8_fwd(buf[p], tau, 256, 1, 0, psi, sub := [])
                acc = [(p, x) for x in sub]
            elif pas == 1:
                p, tw = l >> 5, 32 * w + (l & 31)
                base.r8_fwd(buf[p], ((tw >> 5) << 8) + (tw & 31), 32, 8, tw >> 5, psi, sub := [])
                acc = [(p, x) for x in sub]
            elif pas == 2:
                p, tw = l >> 5, 32 * w + (l & 31)
                base.r8_fwd(buf[p], ((tw >> 2) << 5) + (tw & 3), 4, 64, tw >> 2, psi, sub := [])
                acc = [(p, x) for x in sub]
            else:
                u = 64 * w + l
                for p in range(2):
                    v = [buf[p][4 * u + k] for k in range(4)]
                    acc.extend((p, 4 * u + k) for k in range(4))
                    base.ct(v, 0, 2, psi[N // 4 + u]), base.ct(v, 1, 3, psi[N // 4 + u])
                    base.ct(v, 0, 1, psi[N // 2 + 2 * u]), base.ct(v, 2, 3, psi[N // 2 + 2 * u + 1])
                    for k in range(4):
                        buf[p][4 * u + k] = v[k]
            per[t] = acc
        trace.append(per)
    return buf


def inv_passes(a, ipsi, trace):
    buf = [row[:] for row in a]
    for pas in range(4):
        per = {}
        for t in range(512):
            w, l = t >> 6, t & 63
            acc = []
            if pas == 0:
                u = 64 * w + l
                for p in range(2):
                    v = [buf[p][4 * u + k] for k in range(4)]
                    acc.extend((p, 4 * u + k) for k in range(4))
                    base.gs(v, 0, 1, ipsi[N // 2 + 2 * u]), base.gs(v, 2, 3, ipsi[N // 2 + 2 * u + 1])
                    base.gs(v, 0, 2, ipsi[N // 4 + u]), base.gs(v, 1, 3, ipsi[N // 4 + u])
                    for k in range(4):
                        buf[p][4 * u + k] = v[k]
            elif pas == 1:
                p, tw = l >> 5, 32 * w + (l & 31)
                base.r8_inv(buf[p], ((tw >> 2) << 5) + (tw & 3), 4, 256, tw >> 2, ipsi, sub := [])
                acc = [(p, x) for x in sub]
            elif pas == 2:
                p, tw = l >> 5, 32 * w + (l & 31)
                base.r8_inv(buf[p], ((tw >> 5) << 8) + (tw & 31), 32, 32, tw >> 5, ipsi, sub := [])
                acc = [(p, x) for x in sub]
            else:
                p, tau = t >> 8, t & 255
                base.r8_inv(buf[p], tau, 256, 4, 0, ipsi, sub := [])
                acc = [(p, x) for x in sub]
            per[t] = acc
        trace.append(per)
    return buf


def banks(trace, name):
    worst = 1
    for per in trace:
        nacc = len(per[0])
        for j in range(nacc):
            for w in range(8):
                for half in range(2):
                    lanes = range(64 * w + 32 * half, 64 * w + 32 * half + 32)
                    slots = []
                    for t in lanes:
                        p, x = per[t][j]
                        slots.append((p * N + swz(x)) % 32)
                    worst = max(worst, max(slots.count(s) for s in set(slots)))
    print(f"{name}: worst b64 bank multiplicity per half-wave = {worst}")
    return worst


def wave_local(per, name):
    for t, acc in per.items():
        w = t >> 6
        for p, x in acc:
            if x // 256 != w:
                print(f"{name}: thread {t} (wave {w}) touches element {x} of polynomial {p}")
                return False
    return True


def main():
    rnd = random.Random(2)
    psi = [rnd.randrange(P) for _ in range(N)]
    ipsi = [rnd.randrange(P) for _ in range(N)]
    a = [[rnd.randrange(P) for _ in range(N)] for _ in range(2)]
    tf, ti = [], []
    out = fwd_passes(a, psi, tf)
    assert all(out[p] == base.ref_fwd(a[p], psi) for p in range(2)), "forward passes differ from the stage loop"
    out = inv_passes(a, ipsi, ti)
    assert all(out[p] == base.ref_inv(a[p], ipsi) for p in range(2)), "inverse passes differ from the stage loop"
    for per in tf + ti:  # every element of both polynomials exactly once per pass
        assert sorted(e for acc in per.values() for e in acc) == [(p, x) for p in range(2) for x in range(N)]
    print("index algebra: forward and inverse passes equal the stage loops")
    local = all(wave_local(per, "forward") for per in tf[1:]) and all(wave_local(per, "inverse") for per in ti[:3])
    print("wave-locality: passes B, C and the units stay in the wave's block" if local else "NOT wave-local")
    ok = local and banks(tf, "forward") == 1 and banks(ti, "inverse") == 1
    print("OK" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
