#!/usr/bin/env python3
"""Checks the N = 2048 transform passes of blind_rotate_f64.hip (f64_ntt_fwd2048/inv2048).

1. Index algebra: the four passes (radix-8 on stages 0-2, 3-5, 6-8; two radix-4 units on
   9-10), run with the kernel's thread -> element and twiddle formulas, equal the plain
   stage-by-stage CT / GS loops (random twiddle tables mod a prime, so every index matters).
2. LDS banks: every 64-bit access of a wavefront (64 lanes; gfx950 serves a b64 access per
   half-wave, 64 four-byte banks) through swz() touches 32 distinct double slots mod 32
   per half-wave, for every pass, the slot-per-lane accesses (t + 512k) and both polynomials.
Usage: python3 tools/lds_layouts_f64.py
"""
import random

N, TH, P = 2048, 512, 1000000007


def swz(x):
    c = (x >> 5) & 7
    return x ^ (c << 2) ^ (c & 3)


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


def r8_fwd(buf, base, st, m0, g, psi, acc):
    idx = [base + st * k for k in range(8)]
    acc.extend(idx)
    v = [buf[x] for x in idx]
    for k in range(4):
        ct(v, k, k + 4, psi[m0 + g])
    ct(v, 0, 2, psi[2 * m0 + 2 * g]), ct(v, 1, 3, psi[2 * m0 + 2 * g])
    ct(v, 4, 6, psi[2 * m0 + 2 * g + 1]), ct(v, 5, 7, psi[2 * m0 + 2 * g + 1])
    for j in range(4):
        ct(v, 2 * j, 2 * j + 1, psi[4 * m0 + 4 * g + j])
    for k, x in enumerate(idx):
        buf[x] = v[k]


def r8_inv(buf, base, h0, m, g, ipsi, acc):
    idx = [base + h0 * k for k in range(8)]
    acc.extend(idx)
    v = [buf[x] for x in idx]
    for j in range(4):
        gs(v, 2 * j, 2 * j + 1, ipsi[m + 4 * g + j])
    gs(v, 0, 2, ipsi[m // 2 + 2 * g]), gs(v, 1, 3, ipsi[m // 2 + 2 * g])
    gs(v, 4, 6, ipsi[m // 2 + 2 * g + 1]), gs(v, 5, 7, ipsi[m // 2 + 2 * g + 1])
    for k in range(4):
        gs(v, k, k + 4, ipsi[m // 4 + g])
    for k, x in enumerate(idx):
        buf[x] = v[k]


def passes_fwd(a, psi, trace):
    buf = a[:]
    for pas in range(4):
        per_thread = {}
        for tau in range(256):
            acc = []
            if pas == 0:
                r8_fwd(buf, tau, 256, 1, 0, psi, acc)
            elif pas == 1:
                r8_fwd(buf, ((tau >> 5) << 8) + (tau & 31), 32, 8, tau >> 5, psi, acc)
            elif pas == 2:
                r8_fwd(buf, ((tau >> 2) << 5) + (tau & 3), 4, 64, tau >> 2, psi, acc)
            else:
                for r in range(2):
                    u = tau + 256 * r
                    v = [buf[4 * u + k] for k in range(4)]
                    acc.extend(4 * u + k for k in range(4))
                    ct(v, 0, 2, psi[N // 4 + u]), ct(v, 1, 3, psi[N // 4 + u])
                    ct(v, 0, 1, psi[N // 2 + 2 * u]), ct(v, 2, 3, psi[N // 2 + 2 * u + 1])
                    for k in range(4):
                        buf[4 * u + k] = v[k]
            per_thread[tau] = acc
        trace.append(per_thread)
    return buf


def passes_inv(a, ipsi, trace):
    buf = a[:]
    for pas in range(4):
        per_thread = {}
        for tau in range(256):
            acc = []
            if pas == 0:
                for r in range(2):
                    u = tau + 256 * r
                    v = [buf[4 * u + k] for k in range(4)]
                    acc.extend(4 * u + k for k in range(4))
                    gs(v, 0, 1, ipsi[N // 2 + 2 * u]), gs(v, 2, 3, ipsi[N // 2 + 2 * u + 1])
                    gs(v, 0, 2, ipsi[N // 4 + u]), gs(v, 1, 3, ipsi[N // 4 + u])
                    for k in range(4):
                        buf[4 * u + k] = v[k]
            elif pas == 1:
                r8_inv(buf, ((tau >> 2) << 5) + (tau & 3), 4, 256, tau >> 2, ipsi, acc)
            elif pas == 2:
                r8_inv(buf, ((tau >> 5) << 8) + (tau & 31), 32, 32, tau >> 5, ipsi, acc)
            else:
                r8_inv(buf, tau, 256, 4, 0, ipsi, acc)
            per_thread[tau] = acc
        trace.append(per_thread)
    return buf


def check_banks(trace, name):
    # each pass: the j-th access of every lane is one instruction; check per half-wave
    worst = 1
    for pas, per_thread in enumerate(trace):
        nacc = len(per_thread[0])
        for poly in range(2):
            for w in range(4):  # 4 waves per polynomial
                for j in range(nacc):
                    for half in range(2):
                        lanes = range(64 * w + 32 * half, 64 * w + 32 * half + 32)
                        slots = [(poly * N + swz(per_thread[tau][j])) % 32 for tau in lanes]
                        worst = max(worst, max(slots.count(s) for s in set(slots)))
    print(f"{name}: worst b64 bank multiplicity per half-wave = {worst}")
    return worst


def main():
    rnd = random.Random(1)
    psi = [rnd.randrange(P) for _ in range(N)]
    ipsi = [rnd.randrange(P) for _ in range(N)]
    a = [rnd.randrange(P) for _ in range(N)]
    tf, ti = [], []
    assert passes_fwd(a, psi, tf) == ref_fwd(a, psi), "forward passes differ from the stage loop"
    assert passes_inv(a, ipsi, ti) == ref_inv(a, ipsi), "inverse passes differ from the stage loop"
    for tr in tf + ti:  # every element exactly once per pass
        assert sorted(x for acc in tr.values() for x in acc) == list(range(N))
    assert sorted(swz(x) for x in range(N)) == list(range(N))
    print("index algebra: forward and inverse passes equal the stage loops")
    ok = check_banks(tf, "forward") == 1 and check_banks(ti, "inverse") == 1
    worst = 1
    for k in range(4):  # slot-per-lane phases: x = t + 512 k
        for w in range(8):
            for half in range(2):
                slots = [swz(64 * w + 32 * half + l + 512 * k) % 32 for l in range(32)]
                worst = max(worst, max(slots.count(s) for s in set(slots)))
    print(f"slot-per-lane: worst multiplicity = {worst}")
    assert ok and worst == 1
    print("OK")


if __name__ == "__main__":
    main()
