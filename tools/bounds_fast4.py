"""Per-index worst-case magnitude bounds for the 4-wavefront fast kernel's transforms
(blind_rotate_fast4.hip): radix-4 passes over index bit pairs (b9 b8), (b7 b6), ... (b1 b0)
(forward, Cooley-Tukey) and the reverse (inverse, Gentleman-Sande), signed Montgomery
products (|smul(y, w)| <= |y| (Q/2) / 2^32 + Q/2).  RED lists, per inverse pass, which stage's
sum outputs are reduced (smul by R mod Q).  Asserts every 32-bit value < 2^31, the external
product row sums < 2^63, and the accumulator update window, for every digit shape the kernel is
built for.  Run: python3 tools/bounds_fast4.py [Q]"""
import sys

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 134215681
Qh = Q // 2
LIM = 2 ** 31
RED = {0: None, 1: "B", 2: None, 3: "B", 4: None}   # inverse pass (L5, L4, L3, L2, L1) -> reduced stage


def smul_b(y):
    assert y < LIM, f"smul input {y / Q:.2f}Q"
    return y * Qh / 2 ** 32 + LIM * Q / 2 ** 32


def fwd(b_in, small=False):
    b = list(b_in)
    if small:  # pass 0 from the lookup tables: x0 + T1[x2] +- (T2[x1] + T21[x3]), tables reduced (<= Q/2)
        b = [max(b_in) + 3 * (Qh + 1)] * 1024
    for p in range(1 if small else 0, 5):
        for bit in (9 - 2 * p, 8 - 2 * p):
            m = 1 << bit
            nb = list(b)
            for i in range(1024):
                if not i & m:
                    j = i | m
                    v = smul_b(b[j])
                    nb[i] = nb[j] = b[i] + v
                    assert nb[i] < LIM
            b = nb
    return b


def inv(b_in):
    b = list(b_in)
    for p in range(5):
        for s, bit in enumerate((2 * p, 2 * p + 1)):
            m = 1 << bit
            nb = list(b)
            red = RED[p] == "AB"[s]
            for i in range(1024):
                if not i & m:
                    j = i | m
                    t = b[i] + b[j]
                    assert t < LIM, f"inverse pass {p} stage {s}: {t / Q:.2f}Q"
                    nb[i] = smul_b(t) if red else t
                    nb[j] = smul_b(t)
            b = nb
    return b




def check(dig, logg, fold, split=False):
    """DIG digits of base 2^logg per polynomial; fold = top digit eliminated (C rows); split = the SPLIT
    form: each group reduces its own polynomial's half of the row sum, and A is the sum of two such"""
    dmax = 1 << (logg - 1)
    F = max(fwd([dmax] * 1024))
    if logg <= 7:  # pass 0 from the lookup tables (digits in [-64, 64))
        F = max(F, max(fwd([dmax] * 1024, small=True)))
    nt = dig - 1 if fold else dig          # transformed digits
    rowsum = 2 * nt * F * Qh + (2 * F * Qh if fold else 0)  # C rows kept <= F
    assert rowsum < 2 ** 63
    A = rowsum / 2 ** 32 + Qh                 # sredc of the row sum
    if split:
        A = 2 * (rowsum / 2 / 2 ** 32 + Qh)   # two sredc'd half sums
        assert A < LIM
    S = (2 * A * Qh) / 2 ** 32 + Qh           # monomial combination
    msg = ""
    if fold:
        C0 = smul_b(max(fwd([Qh + 1] * 1024)))    # C = N^-1 NTT(acc)
        Cred = smul_b(C0 + 8 * S)
        assert max(C0, Cred) + 7 * S <= F
        msg = f", C {(max(C0, Cred) + 7 * S) / Q:.3f}Q"
    out = max(inv([S] * 1024))
    assert out < 3 * Q, f"inverse output {out / Q:.3f}Q"
    print(f"Q={Q} dig={dig} logG={logg} fold={fold}{' split' if split else ''}: fwd {F / Q:.3f}Q{msg}, S {S / Q:.3f}Q, "
          f"row sums 2^{rowsum.bit_length() if isinstance(rowsum, int) else __import__('math').log2(rowsum):.1f}, "
          f"inverse out {out / Q:.3f}Q (reductions {RED})  OK")


# the shapes blind_rotate_fast4.hip instantiates (fast4_shape_supported)
for shape in ((4, 7, True), (6, 5, True), (5, 5, False), (3, 9, False)):
    check(*shape)
check(4, 7, True, split=True)  # the SPLIT form (STD128 shape only)
