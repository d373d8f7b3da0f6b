"""GPU: the two-group form of the STD128 blind rotation (k_blind_rotate_fast4<..., SPLIT>).

Batches up to `tfhe_knobs.split4` (default 384) run one ciphertext per 512-thread workgroup with its two
accumulator polynomials on two groups of four wavefronts, which exchange the other column's partial row
sums through LDS each round (the reference's CHES experiment calls EvalBinGate on 256 gates:
CHES-experiments.cpp:30-61).  Checked through the C-ABI against the oracle and against the one-group
kernel (split4 = 0): EvalAcc at 1, 3, 64, 256 and 257 ciphertexts and at both power-of-two a-moduli,
gates at 256 decrypting with valid keys, and the batch limit (385 runs the one-group kernel).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def std128(shared_kat):
    s = shared_kat("STD128")  # the session's shared context
    assert s["ctx"].info().br_kernel == 1 and s["ctx"].knobs()["split4"] == 384
    return s


def _inputs(op, B, seed, amod):
    rs = np.random.default_rng(seed)
    a = rs.integers(0, amod, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    return a, acc


@pytest.mark.parametrize("B", [1, 3, 64])
@pytest.mark.parametrize("amod", [1024, 2048])
def test_split_eval_acc_matches_oracle(std128, B, amod):
    op, ctx, orc = std128["op"], std128["ctx"], std128["orc"]
    a, acc = _inputs(op, B, 800 + B + amod, amod)
    assert np.array_equal(ctx.EvalAcc(a, amod, acc), orc.eval_acc(a, amod, acc))


@pytest.mark.parametrize("B", [256, 384, 385])
def test_split_equals_one_group_form(std128, B):
    op, ctx = std128["op"], std128["ctx"]
    a, acc = _inputs(op, B, 900 + B, 1024)
    two = ctx.EvalAcc(a, 1024, acc)
    with ctx.knobs_set(split4=0):
        one = ctx.EvalAcc(a, 1024, acc)
    assert np.array_equal(two, one)
    idx = [0, B // 2, B - 1]
    assert np.array_equal(two[idx], std128["orc"].eval_acc(a[idx], 1024, acc[idx]))


def test_split_gates_decrypt(oracle):
    """AND / NAND / XOR on 256 pairs (the CHES experiment's batch) with valid keys: decrypting, and equal
    to the oracle on a sample."""
    import tfhe_amd

    op, cp = oracle.params_from_set("STD128"), tfhe_amd.params_from_set("STD128")
    rng = oracle.Rng(44)
    sk, bsk, ksk = oracle.keygen(op, rng)
    ctx = tfhe_amd.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    del bsk, ksk
    try:
        rs = np.random.default_rng(4)
        m1, m2 = rs.integers(0, 2, 256), rs.integers(0, 2, 256)
        c1 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m1])
        c2 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m2])
        for gate, f in (("AND", lambda x, y: x & y), ("NAND", lambda x, y: 1 - (x & y)), ("XOR", lambda x, y: x ^ y)):
            out = ctx.EvalBinGate(gate, c1, c2)
            dec = np.array([oracle.decrypt(op, sk, r, 4, op.q) for r in out])
            assert np.array_equal(dec, f(m1, m2)), gate
            assert np.array_equal(out[[0, 255]], orc.eval_bin_gate(gate, c1[[0, 255]], c2[[0, 255]])), gate
    finally:
        ctx.GPUClean()
        orc.close()
