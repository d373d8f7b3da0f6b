"""Worst-case magnitude bounds for the signed-Montgomery fast blind rotation
(tfhe-gpu_amd/csrc/blind_rotate_fast.hip).  Mirrors the kernel's operation order
and asserts that every 32-bit value stays below 2^31, every 64-bit sum below 2^63,
and that the accumulator update lands in (0, 8Q) before its three conditional
subtractions.  Run: python3 tools/bounds_fast.py [Q]   (default: STD128's Q)."""
import sys

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 134215681
assert Q < 2**27 and Q % 2 == 1
Qh = Q // 2            # |centred Montgomery constant| <= Qh
R = 2**32
LIM32, LIM64 = 2**31, 2**63


def chk32(v, what):
    assert v < LIM32, f"{what}: {v / Q:.2f}Q >= 2^31"
    return v


def sredc(T, what):
    assert T < LIM64, f"{what}: 64-bit sum overflow"
    return chk32(T / R + LIM32 * Q / R, what)   # |m| <= 2^31


def smul(y, what):
    chk32(y, what + " (input)")
    return sredc(y * Qh, what)


# forward: digits |d| <= 64, ten CT stages, all elements share a bound per stage
B = 64
for s in range(10):
    B = chk32(B + smul(B, f"fwd stage {s}"), f"fwd stage {s} out")
Bf = B
# k_blind_rotate_fast2: C = N^-1 NTT(acc) from the centred accumulator (|acc| <= Q/2), then
# C <- C + S per round, reduced (smul by R mod Q) every 8 rounds; C enters the row sums as a
# digit, so it must stay within the forward-output bound used there.
B = Qh + 1
for s in range(10):
    B = chk32(B + smul(B, f"acc fwd stage {s}"), f"acc fwd stage {s} out")
C0 = smul(B, "C init (x N^-1)")
# external product
A64 = sredc(8 * Bf * Qh, "ACC64 row sum")
A32 = 4 * sredc(2 * Bf * Qh, "ACC32 pair")
A = max(A64, A32)
S = sredc(2 * A * Qh, "monomial product")
Cmax = C0
for rnd in range(8):
    Cmax = chk32(Cmax + S, "C + S")
Cred = smul(Cmax, "C reduction")
assert max(C0, Cred) + 7 * S <= Bf, "C used as a digit exceeds the forward bound"


def gs(u, v, red=False, what=""):
    chk32(u + v, what + " sum")
    a = smul(u + v, what + " red") if red else u + v
    return a, smul(u + v, what + " diff")   # |u - v| <= |u| + |v|


# inverse: r0-only pass then three radix-8 passes (x[0], x[4] reduced after stage 2)
x = [S] * 8
for q in range(4):
    x[2 * q], x[2 * q + 1] = gs(x[2 * q], x[2 * q + 1], what="inv L4")
for p in range(3):
    b = max(x)
    x = [b] * 8
    for q in range(4):
        x[2 * q], x[2 * q + 1] = gs(x[2 * q], x[2 * q + 1], what=f"inv pass {p} A")
    for h in range(2):
        x[4 * h], x[4 * h + 2] = gs(x[4 * h], x[4 * h + 2], red=True, what=f"inv pass {p} B")
        x[4 * h + 1], x[4 * h + 3] = gs(x[4 * h + 1], x[4 * h + 3], what=f"inv pass {p} B")
    for r in range(4):
        x[r], x[r + 4] = gs(x[r], x[r + 4], what=f"inv pass {p} C")
    for v in x:
        chk32(v, f"inv pass {p} out")
Sout = max(x)
h1 = Qh + 1
lo = -h1 - Sout + h1 + 4 * Q
hi = Qh + Sout + h1 + 4 * Q
assert 0 < lo and hi < 8 * Q, "acc update out of (0, 8Q)"
print(f"Q={Q}: fwd out {Bf / Q:.3f}Q, ACC64 A {A64 / Q:.3f}Q, ACC32 A {A32 / Q:.3f}Q, "
      f"S {S / Q:.3f}Q, C <= {(max(C0, Cred) + 7 * S) / Q:.3f}Q (pre-reduction {Cmax / Q:.3f}Q), inverse out {Sout / Q:.3f}Q, acc update in [{lo / Q:.2f}Q, {hi / Q:.2f}Q)  OK")
