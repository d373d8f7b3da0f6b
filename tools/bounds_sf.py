"""Worst-case magnitude model of the special-form u64 blind rotations (gen3sf, sf2 in
blind_rotate_generic.hip) for Q = 2^k - c (k = 54; c = 77823, the logQ / arbFunc contexts, and
c = 2^20 - 1, the largest c sf_path_supported admits).

Arithmetic (round 4, device_math.hpp sf_mul): every constant w (twiddle, key, monomial) is stored
as W0 = w and W1 = w 2^32 mod Q (both < Q); a product of ANY unsigned 64-bit a with w is
    a w = a0 W0 + a1 W1  (mod Q),   a0 = a mod 2^32,  a1 = a >> 32
    P   = a0 W0lo + a1 W1lo < 2^65       (the carry out of 64 bits is kept)
    H   = a0 W0hi + a1 W1hi + (P >> 32) + carry 2^32 = S >> 32   (must stay < 2^55)
    r   = (S mod 2^55) + (S >> 55) 2c  < 2^55 + 2^32 2c          (2^55 = 2c mod Q)
All values are unsigned, lazily reduced; a "fold" x -> (x mod 2^k) + (x >> k) c (one mad)
brings any x < 2^64 below 2^k + 2^(64-k) c.  This script walks the kernel's schedule with
the worst-case bound of every element and checks
  * every value (product inputs included) is below 2^64,
  * H < 2^55, so the folded quotient S >> 55 fits the mad's 32-bit multiplier,
  * the offsets kQ of the subtractions (the forward's: the 28Q its inputs carry) keep every difference
    non-negative,
  * the accumulator update lands in [0, Q) after one fold and one conditional subtraction.
Usage: python3 tools/bounds_sf.py   (exit 1 on a violation; run by tests/test_layouts.py)
"""
import sys

K = 54
ok = True


def fail(msg):
    global ok
    print("VIOLATION:", msg)
    ok = False


class Arith:
    def __init__(self, c):
        self.C = c
        self.Q = (1 << K) - c


A = Arith(77823)


def mulw(a):
    """bound of sf_mul(a, W0, W1, 2c) for an input bound a"""
    if a >= 1 << 64:
        fail(f"product input 2^{a.bit_length()} >= 2^64")
    Q = A.Q
    a0, a1 = min(a, (1 << 32) - 1), a >> 32
    w_lo, w_hi = (1 << 32) - 1, (Q - 1) >> 32
    P = a0 * w_lo + a1 * w_lo
    if P >= 1 << 65:
        fail("P needs more than one carry")
    H = a0 * w_hi + a1 * w_hi + (P >> 32)
    if H >= 1 << 55:
        fail("H >= 2^55: the folded quotient would not fit 32 bits")
    return (1 << 55) - 1 + (H >> 23) * 2 * A.C


def fold(x):
    if x >= 1 << 64:
        fail("value >= 2^64")
    return (1 << K) - 1 + (x >> K) * A.C


FWD_OFF = 28   # digits enter the forward transform as r + 28Q (gen3sf: r + 28Q or r + 29Q)


def ct(x, y):
    """x, y: (lower, upper) bounds.  y' = x - v with no offset: the transform's inputs carry FWD_OFF Q,
    and the lower bound of every difference must stay >= 0 (it falls by the product bound per stage)"""
    v = mulw(y[1])
    if x[0] - v < 0:
        fail(f"forward difference may go negative (lower bound {x[0] / A.Q:.2f} Q, product < {v / A.Q:.2f} Q)")
    return (x[0], x[1] + v), (x[0] - v, x[1])


def gs(x, y, fold_sum):
    if y > 10 * A.Q:
        fail(f"inverse offset below the subtrahend bound {y / A.Q:.2f} Q")
    d = x + 10 * A.Q                   # x + 10Q - y
    s = x + y
    return (fold(s) if fold_sum else s), mulw(d)


def ct_ofs(x, y):
    """sf2p's and sf2duo's (round-4) form: y' = x + 3Q - v, inputs r + Q (no lower bound needed)"""
    v = mulw(y[1])
    if v > 3 * A.Q:
        fail("forward offset 3Q below the product bound")
    return (0, x[1] + v), (0, x[1] + 3 * A.Q)


CT = ct


# forward radix-8 (stages (k, k+4), (0,2)(1,3)(4,6)(5,7), (2j, 2j+1)) on uniform input bounds x = (lo, hi)
def fwd_r8(x):
    v = [x] * 8
    for k in range(4):
        v[k], v[k + 4] = CT(v[k], v[k + 4])
    for (a, b) in ((0, 2), (1, 3), (4, 6), (5, 7)):
        v[a], v[b] = CT(v[a], v[b])
    for j in range(4):
        v[2 * j], v[2 * j + 1] = CT(v[2 * j], v[2 * j + 1])
    return v


def fwd_r4(x):
    v = [x] * 4
    for (a, b) in ((0, 2), (1, 3)):
        v[a], v[b] = CT(v[a], v[b])
    for (a, b) in ((0, 1), (2, 3)):
        v[a], v[b] = CT(v[a], v[b])
    return v


def inv_r8(x, fold_stage):
    """GS radix-8; fold_stage[s]: fold the sums written in stage s"""
    v = [x] * 8
    for j in range(4):
        v[2 * j], v[2 * j + 1] = gs(v[2 * j], v[2 * j + 1], fold_stage[0])
    for (a, b) in ((0, 2), (1, 3), (4, 6), (5, 7)):
        v[a], v[b] = gs(v[a], v[b], fold_stage[1])
    for k in range(4):
        v[k], v[k + 4] = gs(v[k], v[k + 4], fold_stage[2])
    return v


def inv_r4(x, fold_stage):
    v = [x] * 4
    for (a, b) in ((0, 1), (2, 3)):
        v[a], v[b] = gs(v[a], v[b], fold_stage[0])
    for (a, b) in ((0, 2), (1, 3)):
        v[a], v[b] = gs(v[a], v[b], fold_stage[1])
    return v


# folds of the kernel (must match blind_rotate_generic.hip gen3sf)
FWD_FOLD_PASS = False       # forward: no folds (growth kQ per stage, 11 stages)
INV_FOLD_UNITS = (False, True)    # inverse radix-4 units: fold the second stage's sums
INV_FOLD_PASS = (False, False, True)   # inverse radix-8 passes C, B: fold the last stage's sums
INV_FOLD_LAST = (False, False, False)  # pass A: none (the accumulator update folds)


DUO_MFULL = True  # sf2duo's factors from the whole 2N-row table (SF2D_MFULL, blind_rotate_generic.hip)


def model(rows, sf2=True, form="sf2"):
    """form: "sf2" / gen3sf (two-level LDS factor tables), "sf2p" (one product per factor with a row of
    the 2N-entry table, no offset: S = fold(sf(A0, F+) + sf(A1, F-))), "duo" (sf2duo: a member sums its own
    polynomial's rows only -- `rows` digits x 1 polynomial -- and its accumulator update adds its own
    column's inverse output and the partner's: acc + own + partner, one fold, one conditional subtraction),
    "sfduo" (round 6, split by NTT half: sf2's offset-free forward on r + 28Q and sf2's inverse folds, element by
    element in sf2's order, with sf2p's one product per factor; the update adds one inverse output, as sf2)."""
    Q = A.Q
    # sf2: digits r + 28Q, r in [-B/2, B/2), |r| <= Q/2 for any base the path admits; gen3sf: r mod Q + 28Q;
    # sf2p, sf2duo: r + Q with the offset in the difference (ct_ofs)
    global CT
    CT = ct_ofs if form in ("sf2p", "duo") else ct
    mfull = form in ("sf2p", "sfduo") or (form == "duo" and DUO_MFULL)
    x = (FWD_OFF * Q - Q // 2, FWD_OFF * Q + Q // 2) if sf2 else (FWD_OFF * Q, (FWD_OFF + 1) * Q)
    if form in ("sf2p", "duo"):
        x = (0, 2 * Q)
    for _ in range(3):
        v = fwd_r8(x)
        x = (min(e[0] for e in v), max(e[1] for e in v))
    v = fwd_r4(x)
    D = max(e[1] for e in v)
    R = mulw(D)
    Ap = rows * (1 if form == "duo" else 2) * R   # rows digits x polynomials per (key, column)
    if mfull:
        S = fold(2 * mulw(Ap))
    else:
        # A0j (X^a' - 1) + A1j (X^-a' - 1) by two LDS table factors per term (sf_mono_pair):
        # sf(sf(A0, T_hi), T_lo) + sf(sf(A1, T_hi'), T_lo') + (10Q - fold(A0 + A1)), the sum folded
        if fold(2 * Ap) > 10 * Q:
            fail("monomial offset 10Q below the folded product sum")
        S = fold(2 * mulw(mulw(Ap)) + 10 * Q)
    x = max(inv_r4(S, INV_FOLD_UNITS))
    x = max(inv_r8(x, INV_FOLD_PASS))
    x = max(inv_r8(x, INV_FOLD_PASS))
    out = max(inv_r8(x, INV_FOLD_LAST))
    print(f"  forward outputs < {D / Q:.1f} Q, products < {R / Q:.3f} Q, sums < {Ap / Q:.2f} Q, "
          f"S < {S / Q:.2f} Q, inverse outputs < {out / Q:.2f} Q")
    acc = (Q - 1) + (2 * out if form == "duo" else out)
    f = fold(acc)
    if f >= 2 * Q:
        fail("accumulator update needs more than one conditional subtraction")
    if form == "duo" and acc >= 1 << 64:
        fail("duo update sum >= 2^64")
    return ok


def sf_mul_model(a, w0, w1, c2):
    """the register-level sequence of device_math.hpp sf_mul (32-bit halves, one carry)"""
    M32, M64 = (1 << 32) - 1, (1 << 64) - 1
    a0, a1 = a & M32, a >> 32
    P1 = a0 * (w0 & M32)
    t = a1 * (w1 & M32) + P1
    P, cy = t & M64, t >> 64
    H = a0 * (w0 >> 32) + (P >> 32)
    H = a1 * (w1 >> 32) + H
    if H >= 1 << 64:
        fail("H overflows its register")
    hh = ((H >> 32) + cy) & M32
    hl = H & M32
    hs = ((hh << 32 | hl) >> 23) & M32          # v_alignbit_b32 hh, hl, 23
    L = ((hl & 0x7FFFFF) << 32) | (P & M32)
    return (L + hs * c2) & M64


def exactness(c, trials=20000):
    """sf_mul_model(a, w, w 2^32 mod Q) = a w mod Q for corner and random a < 2^64, w < Q"""
    import random
    Q = (1 << K) - c
    rng = random.Random(c)
    ws = [0, 1, Q - 1, Q - 2, (1 << 32) - 1, 1 << 32, Q >> 1] + [rng.randrange(Q) for _ in range(64)]
    As = [0, 1, (1 << 64) - 1, (1 << 64) - 2, (1 << 32) - 1, 1 << 32, (1 << 63), Q, 3 * Q]
    bad = 0
    for i in range(trials):
        w = ws[i % len(ws)]
        a = As[i % len(As)] if i < 4 * len(As) * len(ws) else rng.getrandbits(64)
        r = sf_mul_model(a, w, (w << 32) % Q, 2 * c)
        if r % Q != a * w % Q or r >= (1 << 55) + (1 << 32) * 2 * c:
            bad += 1
    if bad:
        fail(f"sf_mul model inexact on {bad} of {trials} products (c = {c})")
    print(f"c = {c}: sf_mul model exact on {trials} products")


def main():
    global A
    good = True
    for c in (77823, (1 << 20) - 1):
        exactness(c)
    for c in (77823, (1 << 20) - 1):
        A = Arith(c)
        for name, digits, sf2, form in (("sf2, C3 (one digit per polynomial)", 1, True, "sf2"),
                                        ("sf2, C5b (two digits)", 2, True, "sf2"),
                                        ("sf2, CHES EvalFunc context (three digits)", 3, True, "sf2"),
                                        ("sf2p, C5b from 512 ciphertexts (two digits)", 2, True, "sf2p"),
                                        ("sf2duo, C5b up to 128 ciphertexts (two digits; test-library A/B form)", 2, True, "duo"),
                                        ("sfduo<1>, C3 up to 128 ciphertexts (one digit)", 1, True, "sfduo"),
                                        ("sfduo<2>, C5b up to 128 ciphertexts (two digits)", 2, True, "sfduo"),
                                        ("gen3sf, 3 digits (TOY logQ 23)", 3, False, "sf2"),
                                        ("gen3sf, 8 digits (the most any context has)", 8, False, "sf2")):
            print(f"c = {c}, {name}")
            good &= model(digits, sf2, form)
    print("OK" if good and ok else "FAILED")
    return 0 if good and ok else 1


if __name__ == "__main__":
    sys.exit(main())
