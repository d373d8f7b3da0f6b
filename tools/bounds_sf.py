"""Worst-case magnitude model of the special-form u64 blind rotation (gen3sf in
blind_rotate_generic.hip) for Q = 2^k - c (k = 54, c = 77823: the logQ / arbFunc contexts).

Arithmetic: every constant w (twiddle, key, monomial) is stored as W0 = w and W1 = w 2^31 mod Q
(both < Q); a product of an unsigned 64-bit a < 2^61 with w is
    a w = a0 W0 + a1 W1  (mod Q),   a0 = a mod 2^31,  a1 = a >> 31 < 2^30
    S   = a0 W0 + a1 W1 < 2^86      (four v_mad_u64_u32, no overflow: checked below)
    r   = (S mod 2^k) + (S >> k) c  < 2^k + 2^32 c   (one more v_mad_u64_u32)
All values are unsigned, lazily reduced; a "fold" x -> (x mod 2^k) + (x >> k) c (one mad)
brings any x < 2^64 below 2^k + 2^(64-k) c.  This script walks the kernel's schedule with
the worst-case bound of every element and checks
  * every product input is below 2^61 (so a1 < 2^30) and every value below 2^64,
  * the partial sums of the product never overflow 64 bits,
  * the offsets kQ of the subtractions keep every difference non-negative,
  * the accumulator update lands in [0, Q) after one fold and one conditional subtraction.
Usage: python3 tools/bounds_sf.py   (exit 1 on a violation; run by tests/test_layouts.py)
"""
import sys

K = 54
C = 77823
Q = (1 << K) - C
IN_MAX = 1 << 61          # product input limit
R_MAX = (1 << K) + (1 << 32) * C  # product output bound
ok = True


def fail(msg):
    global ok
    print("VIOLATION:", msg)
    ok = False


def mulw(a):
    if a >= IN_MAX:
        fail(f"product input 2^{a.bit_length()} >= 2^61")
    a0, a1 = (1 << 31) - 1, (a >> 31)
    w_lo, w_hi = (1 << 32) - 1, (Q >> 32)
    P = a0 * w_lo + a1 * w_lo
    if P >= 1 << 64:
        fail("P overflows 64 bits")
    H = a0 * w_hi + a1 * w_hi + (P >> 32)
    if H >= 1 << K:
        fail("H >= 2^k: the folded quotient would not fit 32 bits")
    return R_MAX


def fold(x):
    if x >= 1 << 64:
        fail("value >= 2^64")
    return (1 << K) + (x >> K) * C


OFF_CT = 2 * Q   # forward: y' = x + 2Q - v
OFF_GS = 9 * Q   # inverse: d = x + 9Q - y


def ct(x, y):
    v = mulw(y)
    if v > OFF_CT:
        fail("forward offset below the product bound")
    return x + v, x + OFF_CT


def gs(x, y, fold_sum):
    if y > OFF_GS:
        fail(f"inverse offset below the subtrahend bound {y / Q:.2f} Q")
    d = x + OFF_GS                     # x + 9Q - y
    s = x + y
    return (fold(s) if fold_sum else s), mulw(d)


# forward radix-8 (stages (k, k+4), (0,2)(1,3)(4,6)(5,7), (2j, 2j+1)) on uniform input bound x
def fwd_r8(x):
    v = [x] * 8
    for k in range(4):
        v[k], v[k + 4] = ct(v[k], v[k + 4])
    for (a, b) in ((0, 2), (1, 3), (4, 6), (5, 7)):
        v[a], v[b] = ct(v[a], v[b])
    for j in range(4):
        v[2 * j], v[2 * j + 1] = ct(v[2 * j], v[2 * j + 1])
    return v


def fwd_r4(x):
    v = [x] * 4
    for (a, b) in ((0, 2), (1, 3)):
        v[a], v[b] = ct(v[a], v[b])
    for (a, b) in ((0, 1), (2, 3)):
        v[a], v[b] = ct(v[a], v[b])
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


def model(rows):
    x = Q                       # digits are canonical (r mod Q)
    for _ in range(3):
        x = max(fwd_r8(x))
    D = max(fwd_r4(x))
    print(f"  forward outputs < {D / Q:.1f} Q")
    A = rows * 2 * mulw(D)      # rows digits x 2 polynomials per (key, column)
    # A0j (X^a' - 1) + A1j (X^-a' - 1) with two LDS table factors per monomial:
    # sf(sf(A, T_hi), T_lo) + (9Q - A) per term, the sum folded
    if A > OFF_GS:
        fail("monomial offset 9Q below the product sum bound")
    S = fold(2 * (mulw(mulw(A)) + OFF_GS))
    print(f"  products < {A / Q:.2f} Q, S < {S / Q:.2f} Q")
    x = max(inv_r4(S, INV_FOLD_UNITS))
    x = max(inv_r8(x, INV_FOLD_PASS))
    x = max(inv_r8(x, INV_FOLD_PASS))
    out = max(inv_r8(x, INV_FOLD_LAST))
    print(f"  inverse outputs < {out / Q:.2f} Q")
    acc = (Q - 1) + out
    f = fold(acc)
    if f >= 2 * Q:
        fail("accumulator update needs more than one conditional subtraction")
    return ok


def main():
    good = True
    for name, digits in (("C3 (one digit per polynomial)", 1), ("C5b (two digits)", 2)):
        print(name)
        good &= model(digits)
    print("OK" if good and ok else "FAILED")
    return 0 if good and ok else 1


if __name__ == "__main__":
    sys.exit(main())
