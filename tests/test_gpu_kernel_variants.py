"""Every retained build of the specialised STD128 blind rotation (tfhe_set_kernel_variant,
DESIGN.md 3.1) equals the CPU oracle bit for bit: the default four-wavefront kernel (60) and the
two cross-check builds of its multi-ciphertext paths, two ciphertexts per wavefront (70) and four
per workgroup (86).  Batch sizes that are not multiples of the per-workgroup ciphertext count
exercise the inactive-ciphertext paths."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = [60, 70, 86]


@pytest.fixture(scope="module")
def setup(oracle):
    import tfhe_amd

    op = oracle.params_from_set("STD128")
    rng = oracle.Rng(11)
    sk, bsk, ksk = oracle.keygen(op, rng)
    ctx = tfhe_amd.BinFHEContextHIP(tfhe_amd.params_from_set("STD128")).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    rs = np.random.default_rng(3)
    B = 7
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    acc[1] = 0
    acc[1, 1, ::2] = op.Q // 8 + 1  # a gate test vector
    ref = {amod: orc.eval_acc(a % amod, amod, acc) for amod in (op.q, 2 * op.N)}
    yield dict(tfhe=tfhe_amd, op=op, ctx=ctx, a=a, acc=acc, ref=ref, sk=sk, orc=orc)
    tfhe_amd.lib().tfhe_set_kernel_variant(0)
    ctx.GPUClean()
    orc.close()


@pytest.mark.parametrize("variant", VARIANTS)
def test_variant_matches_oracle(setup, variant):
    lib = setup["tfhe"].lib()
    assert lib.tfhe_set_kernel_variant(variant) == 0
    assert lib.tfhe_get_kernel_variant() == variant
    try:
        for amod, ref in setup["ref"].items():
            g = setup["ctx"].EvalAcc(setup["a"] % amod, amod, setup["acc"])
            assert np.array_equal(g, ref), (variant, amod)
    finally:
        lib.tfhe_set_kernel_variant(0)


@pytest.mark.parametrize("variant", [60, 70, 86])
def test_variant_full_gates_decrypt(setup, oracle, variant):
    """A NAND batch through the fused gate path on the build, checked against the oracle and by
    decryption (B = 9: ragged for 2 and 4 ciphertexts per workgroup/wavefront)."""
    lib = setup["tfhe"].lib()
    op, sk = setup["op"], setup["sk"]
    rng = oracle.Rng(100 + variant)
    m1 = np.array([0, 1, 0, 1, 1, 0, 1, 0, 1])
    m2 = np.array([0, 0, 1, 1, 1, 1, 0, 0, 1])
    c1 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m1])
    c2 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m2])
    assert lib.tfhe_set_kernel_variant(variant) == 0
    try:
        g = setup["ctx"].EvalBinGate("NAND", c1, c2)
    finally:
        lib.tfhe_set_kernel_variant(0)
    assert np.array_equal(g, setup["orc"].eval_bin_gate("NAND", c1, c2))
    dec = [oracle.decrypt(op, sk, r, 4, op.q) for r in g]
    assert dec == [1 - (int(x) & int(y)) for x, y in zip(m1, m2)]


def test_unknown_variant_is_rejected(setup):
    lib = setup["tfhe"].lib()
    assert lib.tfhe_set_kernel_variant(12345) != 0
    assert lib.tfhe_get_kernel_variant() == 60 or lib.tfhe_get_kernel_variant() > 0
