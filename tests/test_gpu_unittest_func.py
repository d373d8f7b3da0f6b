"""The reference's own decrypt-level assertions for the function-evaluation path
(src/binfhe/unittest/UnitTestFunc.cpp), run through the vector API on the GPU with keys
from the oracle's keygen.  Each TEST's loop over inputs becomes one batch.  The
timeOptimization variants (EvalSignFuncTime, EvalDigitDecompTime) are the same
assertions on a context the reference GPU path rejects (binfhecontext.cpp:350-353), so
only the space variants run.  Bit-exactness against the oracle is checked alongside.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _setup(oracle, arb, logQ, seed):
    import tfhe_amd as capi

    op = oracle.params_from_logq("TOY", arb, logQ, 0, 0, 0)
    cp = capi.params_from_logq("TOY", arb, logQ, 0, 0, 0)
    rng = oracle.Rng(seed)
    sk, bsk, ksk = oracle.keygen(op, rng)
    ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    return op, ctx, sk, rng, oracle.Oracle(op, bsk, ksk)


def test_eval_arb_func(oracle):
    """UnitTestFunc.cpp:44-68: GenerateBinFHEContext(TOY, true, 12), cube LUT over p."""
    op, ctx, sk, rng, orc = _setup(oracle, True, 12, 41)
    p = ctx.GetMaxPlaintextSpace()

    def fp(m, p1):
        return (m * m * m) % p1 if m < p1 else ((m - p1 // 2) ** 3) % p1

    iv = op.q // p  # GenerateLUTviaFunction (binfhecontext.cpp:280-301)
    lut = np.array([fp(i // iv, p) * iv for i in range(op.q)], dtype=np.uint64)
    ct = np.stack([oracle.encrypt(op, rng, sk, i % p, p, op.q) for i in range(p)])
    out = ctx.EvalFunc(ct, lut)
    assert np.array_equal(out, orc.eval_func(ct, lut))
    assert [oracle.decrypt(op, sk, r, p, op.q) for r in out] == [fp(i, p) for i in range(p)]
    ctx.GPUClean(), orc.close()


def test_eval_floor_func(oracle):
    """UnitTestFunc.cpp:71-93: TOY, logQ 12, EvalFloor(ct, 1) over p/2-3 .. p/2+4."""
    op, ctx, sk, rng, orc = _setup(oracle, False, 12, 42)
    p = ctx.GetMaxPlaintextSpace()
    ms = list(range(p // 2 - 3, p // 2 + 5))
    ct = np.stack([oracle.encrypt(op, rng, sk, m % p, p, op.q) for m in ms])
    out = ctx.EvalFloor(ct, op.q, 1)
    assert np.array_equal(out, orc.eval_floor(ct, op.q, 1))
    assert [oracle.decrypt(op, sk, r, p // 2, op.q) for r in out] == [m // 2 for m in ms]
    ctx.GPUClean(), orc.close()


def test_eval_sign_func_space(oracle):
    """UnitTestFunc.cpp:117-137: TOY, logQ 29, sign of p*factor/2 + i - 3, Q = 2^29."""
    op, ctx, sk, rng, orc = _setup(oracle, False, 29, 43)
    Q = 1 << 29
    factor = 1 << int(29 - math.log2(op.q))
    p = ctx.GetMaxPlaintextSpace()
    ms = [p * factor // 2 + i - 3 for i in range(8)]
    ct = np.stack([oracle.encrypt(op, rng, sk, m, p * factor, Q) for m in ms])
    out = ctx.EvalSign(ct, Q)
    assert np.array_equal(out, orc.eval_sign(ct, Q))
    assert [oracle.decrypt(op, sk, r, 2, op.q) for r in out] == [int(i >= 3) for i in range(8)]
    ctx.GPUClean(), orc.close()


def test_eval_digit_decomp_space(oracle):
    """UnitTestFunc.cpp:198-264: TOY, logQ 29, every digit of the decomposition of
    P/2-3 .. P/2+4 decrypts to the reference's expected digit."""
    op, ctx, sk, rng, orc = _setup(oracle, False, 29, 44)
    Q = 1 << 29
    factor = 1 << int(math.log2(Q) - math.log2(op.q))
    p_basic = ctx.GetMaxPlaintextSpace()
    P = p_basic * factor
    st = P // 2 - 3
    ms = list(range(st, st + 8))
    ct = np.stack([oracle.encrypt(op, rng, sk, m, P, Q) for m in ms])
    digits, moduli = ctx.EvalDecomp(ct, Q)
    d_c, mods_c = orc.eval_decomp(ct, Q)
    assert moduli == mods_c and np.array_equal(digits, d_c)
    nd = int(math.ceil(math.log(factor) / math.log(p_basic)) + 1)
    assert digits.shape[1] == nd
    msb = lambda x: int(x).bit_length()  # noqa: E731  (GetMSB)
    for k, i in enumerate(ms):
        for j in range(nd):
            pd = p_basic if j < nd - 1 else 1 << (msb(P - 1) % msb(p_basic - 1))
            # digits 0..nd-2 are mod q; the last keeps the modulus the floors left it
            # (binfhe-base-scheme.cpp:1067-1086), and Decrypt uses the ciphertext's own
            got = oracle.decrypt(op, sk, digits[k, j], pd, moduli[j])
            if i < st + 3:
                want = 13 + i - st if j == 0 else (0 if j == nd - 1 else 15)
            else:
                want = i - (st + 3) if j == 0 else (1 if j == nd - 1 else 0)
            assert got == want, (i, j)
    ctx.GPUClean(), orc.close()
