"""GPU: the special-form kernels at every digit count a Q = 2^54 - c context reaches.

sf2 is built for 1, 2 and 3 transformed digits (2 also as sf2p, two ciphertexts per 1024-thread
workgroup with the whole monomial table in their shared LDS -- the default above the duo batches) (3: the CHES-experiments.cpp EvalFunc context,
GenerateBinFHEContext(STD128, true, 12, 0, GINX, false, 1 << 18) -- baseG 2^18, no thrown digit),
gen3sf takes more (TOY logQ 29: 4, tests/test_gpu_unittest_func.py) and is the cross-check of all
(knob sf2 = 0).  Per context: EvalAcc on 5 ciphertexts bit-exact against the oracle, and 64
ciphertexts equal on sf2 and gen3sf.  Keys: Appendix B splitmix64 keys (the session's shared contexts).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CONTEXTS = {  # name: the shared context (conftest.SHARED_SPECS), transformed digits
    "C3_arb_logQ12_thr1": ("ARB12", 1),
    "C5b_logQ23_thr1": ("LOGQ23", 2),
    "CHES_func_baseG18": ("CHES18", 3),
}


@pytest.fixture(scope="module", params=list(CONTEXTS))
def sfctx(request, shared_kat):
    name, digits = CONTEXTS[request.param]
    s = shared_kat(name)
    op, cp, ctx = s["op"], s["cp"], s["ctx"]
    assert cp.digitsG - cp.numDigitsToThrow == digits and cp.Q == (1 << 54) - 77823
    assert ctx.info().br_kernel == 5  # TFHE_BR_SF
    return op, ctx, s["orc"]


def _inputs(op, B, seed):
    rs = np.random.default_rng(seed)
    return (rs.integers(0, 2 * op.N, (B, op.n), dtype=np.uint64),
            rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64))


def test_sf2_eval_acc_matches_oracle(sfctx):
    op, ctx, orc = sfctx
    a, acc = _inputs(op, 5, 11)
    out = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(out.reshape(5, -1), orc.eval_acc(a, 2 * op.N, acc).reshape(5, -1))


def test_sf2_equals_gen3sf(sfctx):
    op, ctx, _ = sfctx
    a, acc = _inputs(op, 64, 12)
    with ctx.knobs_set(duo=0):
        one = ctx.EvalAcc(a, 2 * op.N, acc)
    with ctx.knobs_set(sf2=0):
        ref = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(one, ref)


@pytest.mark.parametrize("B", [511, 512, 513])
def test_sf2_pair_form_equals_one_ciphertext_form(sfctx, B):
    """sf2p (default from 512 ciphertexts) = sf2 with one ciphertext per workgroup (knob sf2p = 0), odd
    batches included (the last workgroup's second half repeats its neighbour and does not store)."""
    op, ctx, orc = sfctx
    a, acc = _inputs(op, B, 13 + B)
    with ctx.knobs_set(duo=0):
        two = ctx.EvalAcc(a, 2 * op.N, acc)
        with ctx.knobs_set(sf2p=0):
            one = ctx.EvalAcc(a, 2 * op.N, acc)
    assert np.array_equal(two, one)
    assert np.array_equal(two[-1:].reshape(1, -1), orc.eval_acc(a[-1:], 2 * op.N, acc[-1:]).reshape(1, -1))
