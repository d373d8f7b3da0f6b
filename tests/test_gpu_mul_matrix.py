"""CiphertextMulMatrix (lwe-operation.cu:50-137; binfhecontext.cpp:319-321) on the GPU.

The reference computes out[c] = sum_k matrix[k][c] * ct[k] as an FP64 DGEMM followed by
fmod (exact only while every |sum| < 2^53 and non-negative); the HIP kernel sums exactly
and reduces into [0, modulus).  Where the reference is exact the two agree, which the
first test checks on examples/GEMM.cpp's own configuration (STD128 arbFunc logQ=12
throw=1, modulus qKS = 2^35, matrix entries in [0, 64), its bit-compare loop at
GEMM.cpp:110-120), against both the reference's FP64 formula and an exact integer product.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def arb12(oracle):
    import tfhe_amd as capi

    op = oracle.params_from_logq("STD128", True, 12, 0, 0, 1)
    cp = capi.params_from_logq("STD128", True, 12, 0, 0, 1)
    bsk, ksk = oracle.kat_keys(op, oracle.Rng(51))
    ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    yield op, ctx
    ctx.GPUClean()


def test_gemm_example_config(arb12):
    op, ctx = arb12
    qks = op.qKS
    rs = np.random.default_rng(8)
    K, cols = 1024, 192
    ct = rs.integers(0, qks, (K, op.n + 1), dtype=np.uint64)
    mat = rs.integers(0, 1 << 6, (K, cols), dtype=np.int64)
    out = ctx.CiphertextMulMatrix(ct, mat, qks)
    exact = (mat.T @ ct.astype(np.int64)) % qks  # sums < 2^35 * 2^6 * 2^10 = 2^51: no int64 overflow
    assert np.array_equal(out, exact.astype(np.uint64))
    fp = np.fmod(mat.T.astype(np.float64) @ ct.astype(np.float64), float(qks)).astype(np.uint64)  # CPUGEMM
    assert np.array_equal(out, fp)


def test_exact_beyond_fp64_range(arb12):
    """Negative coefficients and sums far above 2^53: exact integer semantics."""
    op, ctx = arb12
    rs = np.random.default_rng(9)
    K, cols, mod = 7, 5, (1 << 54) - 77823
    ct = rs.integers(0, mod, (K, op.n + 1), dtype=np.uint64)
    mat = rs.integers(-(1 << 62), 1 << 62, (K, cols), dtype=np.int64)
    mat[0, 0] = np.iinfo(np.int64).min
    out = ctx.CiphertextMulMatrix(ct, mat, mod)
    for c in range(cols):
        for w in (0, 1, op.n // 2, op.n):
            want = sum(int(mat[k, c]) * int(ct[k, w]) for k in range(K)) % mod
            assert int(out[c, w]) == want, (c, w)


def test_errors(arb12):
    import tfhe_amd as capi

    op, ctx = arb12
    ct = np.zeros((0, op.n + 1), dtype=np.uint64)
    with pytest.raises((capi.TfheError, ValueError)):
        ctx.CiphertextMulMatrix(ct, np.zeros((0, 3), dtype=np.int64), 1 << 35)
    ct = np.zeros((2, op.n + 1), dtype=np.uint64)
    with pytest.raises((capi.TfheError, ValueError)):
        ctx.CiphertextMulMatrix(ct, np.zeros((3, 3), dtype=np.int64), 1 << 35)  # rows != ciphertexts


@pytest.mark.parametrize("mod", [(1 << 35), (1 << 63) + 29, (1 << 64) - 59])
def test_extreme_entries(arb12, mod):
    """INT64_MIN / INT64_MAX entries and u64-wide ciphertext words: operands are reduced
    into [0, modulus) first, so the sum is exact even where K products of 2^127 would
    overflow an unreduced 128-bit accumulator.  Per-term reduction is taken
    when K (modulus-1)^2 >= 2^128 (the two large moduli)."""
    op, ctx = arb12
    rs = np.random.default_rng(10)
    K, cols = 9, 4
    ct = rs.integers(0, np.iinfo(np.uint64).max, (K, op.n + 1), dtype=np.uint64, endpoint=True)
    ct[0, :] = np.iinfo(np.uint64).max
    mat = rs.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, (K, cols), dtype=np.int64, endpoint=True)
    mat[:, 0] = np.iinfo(np.int64).min
    mat[:, 1] = np.iinfo(np.int64).max
    out = ctx.CiphertextMulMatrix(ct, mat, mod)
    for c in range(cols):
        for w in (0, 1, op.n // 3, op.n):
            want = sum(int(mat[k, c]) * int(ct[k, w]) for k in range(K)) % mod
            assert int(out[c, w]) == want, (c, w)


def test_reference_fixtures(arb12):
    """Against the reference's own CPU CiphertextMulMatrix (tests/golden/ref_vectors.json mm_*: outputs of
    CPUGEMM, examples/GEMM.cpp:30-56, the function the reference's GEMM example checks its GPU result
    against, compiled from that file by oracle/Makefile.ref and run by tools/gen_golden.py; its FP64 sum
    + fmod + static_cast<uint64_t> semantics equal lwe-operation.cu:79-125's, and the numpy restatement
    refvec.mulmatrix_reference reproduces them bit for bit: tests/test_oracle_ref_vectors.py).
      mm_gemm     GEMM.cpp's config (K = 1024, entries [0, 64)): every sum exact -> equal to the fixture.
      mm_negative entries in [-64, 64): the reference's fmod keeps a negative sum's sign and the cast
                  wraps it to 2^64 - |r| (outside [0, qKS)); the kernel returns the residue qKS - |r|.
      mm_above53  sums up to 2^80: the reference's FP64 sum rounds; the kernel is exact.
    The kernel equals the exact product everywhere and the reference wherever the reference is exact."""
    import refvec

    op, ctx = arb12
    data = refvec.load()
    for name in ("mm_gemm", "mm_negative", "mm_above53"):
        c = refvec.case(name, data)
        x = refvec.inputs(c, data["fixtures"])
        m = c["args"]["modulus"]
        out = ctx.CiphertextMulMatrix(x["in"], x["matrix"], m)
        ref = refvec.mulmatrix_reference(x["in"], x["matrix"], m)
        if name == "mm_gemm":
            refvec.check(c, out.ravel(), {})
            continue
        exact = refvec.mulmatrix_exact(x["in"], x["matrix"], m)
        assert np.array_equal(out, exact), name
        if name == "mm_negative":
            neg = ref >= np.uint64(1 << 63)
            assert neg.any() and (~neg).any()
            with np.errstate(over="ignore"):
                assert np.array_equal(out[neg], ref[neg] + np.uint64(m))  # (2^64 - |r|) + qKS mod 2^64
            assert np.array_equal(out[~neg], ref[~neg])
        else:
            assert (out != ref).mean() > 0.5, "the reference's FP64 sums must round here"
