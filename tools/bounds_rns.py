"""Worst-case magnitude model of the RNS blind rotation (blind_rotate_rns.hip).

Every residue is a signed int32 (signed Montgomery, R = 2^32, prime p < 2^26).  This script
walks the kernel's exact schedule -- digit -> forward transform (radix-8 passes A, B, C on
stages 0-8, radix-4 units on stages 9-10), products, monomial product, inverse transform
(units, passes C, B, A), reduction of the final outputs -- with the worst-case bound of every
element, and checks that
  * every int32 value stays below 2^31 (no wrap),
  * every Montgomery input T stays below 2^62,
  * the inverse outputs handed to the CRT are below p (canonicalised by one conditional add).
It also checks the CRT range: 4 dG2 N max|digit| max|key| < M / 2 for the configurations.
Usage: python3 tools/bounds_rns.py  (exit 1 on a violation; run by tests/test_layouts.py)
"""
import sys

from fractions import Fraction as F

P_MAX = (1 << 26) - 1      # primes are p = 1 (mod 4096) below 2^26
HALF = F(P_MAX, 2)         # centred constants (twiddles, keys, monomials): |w| <= p/2
LIM32 = 1 << 31


def sredc(T):
    """|sredc(T)| <= |T| / 2^32 + p/2 (m = lo32(T) q^-1 is a signed 32-bit value)."""
    assert T < (1 << 62), "Montgomery input too large"
    return F(T) / (1 << 32) + HALF


def smul(x):
    return sredc(x * HALF)


ok = True


def check(name, v):
    global ok
    if v >= LIM32:
        print(f"OVERFLOW {name}: {float(v):.4g} >= 2^31")
        ok = False


# the radix-8 cores of the kernel: element k's bound after the three stages
def fwd_r8(x):
    v = list(x)
    for k in range(4):                      # stage 1: (k, k+4)
        t = smul(v[k + 4]); v[k], v[k + 4] = v[k] + t, v[k] + t
    for (a, b) in ((0, 2), (1, 3), (4, 6), (5, 7)):
        t = smul(v[b]); v[a], v[b] = v[a] + t, v[a] + t
    for j in range(4):
        t = smul(v[2 * j + 1]); v[2 * j], v[2 * j + 1] = v[2 * j] + t, v[2 * j] + t
    return v


def fwd_r4(x):
    v = list(x)
    for (a, b) in ((0, 2), (1, 3)):
        t = smul(v[b]); v[a], v[b] = v[a] + t, v[a] + t
    for (a, b) in ((0, 1), (2, 3)):
        t = smul(v[b]); v[a], v[b] = v[a] + t, v[a] + t
    return v


def inv_r8(x, red):
    """GS radix-8 (stages h0, 2h0, 4h0); red: element indices reduced (smul by R mod p) at the end."""
    v = list(x)
    for j in range(4):
        a, b = 2 * j, 2 * j + 1
        v[a], v[b] = v[a] + v[b], smul(v[a] + v[b])
    for (a, b) in ((0, 2), (1, 3), (4, 6), (5, 7)):
        v[a], v[b] = v[a] + v[b], smul(v[a] + v[b])
    for k in range(4):
        v[k], v[k + 4] = v[k] + v[k + 4], smul(v[k] + v[k + 4])
    for k in range(8):
        check("inverse radix-8 output", v[k])
        if k in red:
            v[k] = smul(v[k])
    return v


def inv_r4(x, red):
    v = list(x)
    for (a, b) in ((0, 1), (2, 3)):
        v[a], v[b] = v[a] + v[b], smul(v[a] + v[b])
    for (a, b) in ((0, 2), (1, 3)):
        v[a], v[b] = v[a] + v[b], smul(v[a] + v[b])
    for k in range(4):
        check("inverse radix-4 output", v[k])
        if k in red:
            v[k] = smul(v[k])
    return v


# reductions of the kernel (must match blind_rotate_rns.hip RED_* constants)
RED_UNITS = (0,)          # after the radix-4 units of the inverse: element 0 (the pure sum)
RED_PASS = (0,)           # after inverse passes C and B: element 0
RED_FINAL = (0, 1, 2, 3)  # after pass A: the sum-chain outputs, so that every output is < p


def model(max_digit, rows):  # rows = digits per polynomial
    x = [F(max_digit)] * 8
    for _ in range(3):                      # passes A, B, C
        x = [max(fwd_r8(x))] * 8
    x = [max(fwd_r4(x[:4]))] * 8            # stages 9-10
    for v in x:
        check("forward output", v)
    D = x[0]
    # products: per digit, the two polynomials' terms D * K per (key, column) in int64, one
    # sredc per digit, digits summed in int32
    A = rows * sredc(2 * D * HALF)
    check("product sum", A)
    # monomial: A00 mp + A10 mn
    S = sredc(2 * A * HALF)
    x = inv_r4([S] * 4, RED_UNITS)
    x = [max(x)] * 8
    x = inv_r8(x, RED_PASS)                 # pass C
    x = [max(x)] * 8
    x = inv_r8(x, RED_PASS)                 # pass B
    x = [max(x)] * 8
    x = inv_r8(x, RED_FINAL)                # pass A
    out = max(x)
    if out >= P_MAX:
        print(f"final output {float(out):.4g} not below p")
        return False
    return True


# (name, N, dG2, rows per digit and key column (= 2: both polynomials), digits, logG, thr, logQ)
CONFIGS = [
    ("C3 arbFunc logQ=12 throw=1", 2048, 2, 1, 27, 1, 54),
    ("C5b logQ=23 throw=1", 2048, 4, 2, 18, 1, 54),
]


def crt_ok(N, dG2, digits, logG, thr, logQ, M):
    Q = (1 << logQ)
    B = 1 << logG
    # top digit after thr thrown and digits-1 kept ones of a centred |c| < Q/2
    top = (Q // 2) // (B ** (thr + digits - 1)) + 2
    maxd = max(B // 2, top)
    bp = dG2 * N * maxd * (Q // 2)
    return 4 * bp < M // 2, maxd


def main():
    primes = []
    p = ((1 << 26) // 4096) * 4096 + 1
    while len(primes) < 4:
        p -= 4096
        if p < (1 << 26) and all(p % d for d in range(2, int(p ** 0.5) + 1)):
            primes.append(p)
    M = 1
    for q in primes:
        M *= q
    print("primes", primes, f"M = 2^{M.bit_length() - 1}.x")
    good = True
    for name, N, dG2, digits, logG, thr, logQ in CONFIGS:
        c, maxd = crt_ok(N, dG2, digits, logG, thr, logQ, M)
        m = model(maxd, digits)
        print(f"{name}: max digit 2^{maxd.bit_length() - 1}, CRT range {'ok' if c else 'TOO SMALL'}, "
              f"int32 bounds {'ok' if m and ok else 'VIOLATED'}")
        good &= c and m and ok
    return 0 if good else 1


if __name__ == "__main__":
    sys.exit(main())
