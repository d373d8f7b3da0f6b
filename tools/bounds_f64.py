"""Worst-case magnitude walk of the wave-local FP64 blind rotation (k_blind_rotate_f64w,
blind_rotate_f64.hip) for every reducing parameter set (RED: 2^40 <= Q < 2^50, i.e. STD128Q and
STD128Q_OPT, Q = 2^50 - 2^14 + 1).  Every value is an integer held in a double, so every sum and
every fmodmul operand must stay below 2^53.

fmodmul(a, b), |a| <= A, |b| <= Bw:
    h = RN(ab)            |h| <= RN(A Bw)
    l = fma(a, b, -h)     exact, |l| <= ulp(A Bw) / 2
    t = RN(h Qinv)        |t - h/Q| <= |h/Q| |eps| + ulp(|h/Q|) / 2,   eps = RN(1/Q) Q - 1 (exact for this Q)
    q = rint(t)           |q - h/Q| <= 1/2 + that
    r = fma(-q, Q, h)     exact (an integer below 2^52)
    out = r + l           exact, |out| <= (1/2 + dt) Q + ulp(A Bw) / 2
fred(x) = fma(-rint(x Qinv), Q, x): the same with l = 0 and h = x.

The walk follows the kernel's schedule element by element (N = 2048, one polynomial):
  forward  CT stages len = 1024 .. 1 (passes A: 1024-256, B: 128-32, C: 16-4, units: 2, 1),
           one fred after pass B;
  products rows D (forward outputs, LD of them) and C' (|C'| <= fred bound) times keys (<= Q/2),
           2 LD + 2 rows summed per ternary key;
  monomial MT 3: W = fmodmul(T_hi, T_lo) - 1, sv = fred(fmodmul(A0, W+) + fmodmul(A1, W-));
  inverse  GS stages len = 1 .. 1024 (units 1, 2 -> fred on x & 3 in {0, 1}; passes C (4-16) and
           B (32-128) -> fred on every element; pass A 256-1024 none).  Round 2 reduced only the sums
           (k < 4) of passes C and B: a pass-A thread whose 8 inputs are all unreduced products then
           sums to 12 Q > 2^53 in the worst case (--round2 shows that walk);
  update   c + r (|c| <= Q/2) then fred.
Exit 1 if any bound reaches 2^53.
"""
import math
import sys
from fractions import Fraction

LIM = 2.0 ** 53
N = 2048


def ulp(x):
    return 2.0 ** (math.floor(math.log2(x)) - 52) if x > 0 else 0.0


class Arith:
    def __init__(self, Q):
        self.Q = Q
        qinv = 1.0 / Q  # RN(1/Q)
        self.eps = abs(float(Fraction(qinv) * Q - 1))
        self.worst = 0.0
        self.where = ""

    def note(self, x, where):
        if x > self.worst:
            self.worst, self.where = x, where
        return x

    def fmodmul(self, A, Bw, where=""):
        self.note(A, where + " (fmodmul operand)")
        P = A * Bw
        h = P * (1 + 2.0 ** -53)
        hq = h / self.Q
        dt = hq * self.eps + ulp(hq * (1 + self.eps)) / 2
        return (0.5 + dt) * self.Q + ulp(P) / 2

    def fred(self, X, where=""):
        self.note(X, where + " (fred operand)")
        xq = X / self.Q
        dt = xq * self.eps + ulp(xq * (1 + self.eps)) / 2
        return (0.5 + dt) * self.Q

    def add(self, *xs, where=""):
        return self.note(sum(xs), where)


def forward(ar, x0, reduce_after_len=32):
    Qh = ar.Q / 2
    X = x0
    ln = N // 2
    while ln >= 1:
        X = ar.add(X, ar.fmodmul(X, Qh, f"forward len {ln}"), where=f"forward len {ln}")
        if ln == reduce_after_len:
            X = ar.fred(X, f"forward len {ln}")
        ln //= 2
    return X


ROUND2 = "--round2" in sys.argv


def inverse(ar, s0):
    Qh = ar.Q / 2
    B = [s0] * N
    if ROUND2:
        red = {2: lambda x: (x & 3) in (0, 1), 16: lambda x: not (x >> 4) & 1, 128: lambda x: not (x >> 7) & 1}
    else:
        red = {2: lambda x: (x & 3) in (0, 1), 16: lambda x: True, 128: lambda x: True}
    ln = 1
    while ln < N:
        nb = B[:]
        for i in range(N):
            if i & ln:
                continue
            a, b = B[i], B[i + ln]
            s = ar.add(a, b, where=f"inverse len {ln}")
            nb[i] = s
            nb[i + ln] = ar.fmodmul(s, Qh, f"inverse len {ln}")
        B = nb
        if ln in red:
            B = [ar.fred(v, f"inverse len {ln}") if red[ln](x) else v for x, v in enumerate(B)]
        ln *= 2
    return max(B)


def walk(Q, LD):
    ar = Arith(Q)
    Qh = Q / 2
    F = ar.fred(Qh)  # a fred'ed value
    d_out = max(forward(ar, 2.0 ** 24), forward(ar, Qh))  # digits; C' prologue and the WRAP digit (<= Q/2)
    cx = ar.fred(ar.add(F, d_out))  # C' with the WRAP correction added
    A = ar.add(*([ar.fmodmul(d_out, Qh, "products")] * (2 * LD) + [ar.fmodmul(cx, Qh, "products")] * 2),
               where="product sums")
    W = ar.fmodmul(Qh, Qh, "monomial table product") + 1
    sv = ar.fred(ar.add(ar.fmodmul(A, W, "monomial"), ar.fmodmul(A, W, "monomial"), where="monomial sum"))
    ar.fred(ar.add(F, sv, where="C' update"))
    r = inverse(ar, sv)
    ar.fred(ar.add(Qh, r, where="accumulator update"), "accumulator update")
    return ar, d_out, A, r


def main():
    ok = True
    for name, Q, LD in (("STD128Q / STD128Q_OPT", 2 ** 50 - 2 ** 14 + 1, 1),):
        ar, d_out, A, r = walk(Q, LD)
        print(f"{name}: Q = 2^{math.log2(Q):.6f}, |RN(1/Q) Q - 1| = 2^{math.log2(ar.eps):.1f}")
        print(f"  forward outputs <= {d_out / Q:.3f} Q, product sums <= {A / Q:.3f} Q, inverse outputs <= {r / Q:.3f} Q")
        print(f"  largest operand or sum: {ar.worst / Q:.3f} Q = 2^{math.log2(ar.worst):.4f} at {ar.where}"
              f"  {'OK' if ar.worst < LIM else 'OVER 2^53'}")
        ok &= ar.worst < LIM
    print("OK" if ok else "FAIL")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
