"""The C restatement (oracle/) against the REFERENCE's vector-API outputs.

tests/golden/ref_vectors.json was written by tools/gen_golden.py from oracle/_ref/ref_kat: the
reference's own OpenFHE code (/root/reference, compiled by oracle/Makefile.ref), its vector
BinFHEScheme functions unchanged, the seven GPU symbols served by its own CPU functions.  Every
case is re-run here through the oracle on the same regenerated inputs: all 8 gates, EvalAcc and
MKMSwitch at the boundary (three a-moduli, two output moduli), EvalFunc with the reference's
cube LUT and with per-ciphertext LUTs, EvalFloor, and EvalSign / EvalFloor / EvalDecomp on the
two BASELINE C5 contexts (STD128Q and logQ = 23, Qin = 2^23).
"""
import numpy as np
import pytest

import refvec

DATA = refvec.load()
_ctx_cache = {}


def oracle_for(oracle, c):
    key = (c["ctx"], c["keys"])
    if key not in _ctx_cache:
        for k in list(_ctx_cache):  # one context alive at a time (STD128Q keys are 2.7 GB)
            _ctx_cache.pop(k).close()
        p = refvec.params(oracle, c["ctx"])
        bsk, ksk = refvec.keys(c, p)
        _ctx_cache[key] = oracle.Oracle(p, bsk, ksk)
    return _ctx_cache[key]


# the larger batches written for the multi-device drop-in (tests/test_gpu_dropin.py) repeat contexts and
# operations already pinned here at B = 4; only the cheap gate batch runs on the CPU suite
MULTIDEV_ONLY = {"arb12_func_cube_b7", "c5a_std128q_sign_b7"}
BOOTSTRAP_CASES = [c["name"] for c in DATA["cases"] if c["op"] != "mulmatrix" and c["name"] not in MULTIDEV_ONLY]
MM_CASES = [c["name"] for c in DATA["cases"] if c["op"] == "mulmatrix"]


@pytest.mark.parametrize("name", BOOTSTRAP_CASES)
def test_oracle_matches_reference_vector_api(oracle, name):
    c = refvec.case(name, DATA)
    o = oracle_for(oracle, c)
    out, extra = refvec.run(c, DATA["fixtures"], refvec.OracleOps(o))
    refvec.check(c, out, extra)


def test_vector_equals_single_in_reference():
    """The generator ran every case through the reference's single-ciphertext API too."""
    for c in DATA["cases"]:
        if c["op"] != "mulmatrix":  # (CiphertextMulMatrix has no single-ciphertext form)
            assert c["single_fnv"] == c["vector"]["fnv"], c["name"]


def test_cube_lut_is_the_reference_lut():
    """helpers.cube_lut == BinFHEContext::GenerateLUTviaFunction(x^3 mod 8) on the arbFunc logQ = 12
    context (binfhecontext.cpp:280-301; time-estimate.cpp:67-76)."""
    from helpers import cube_lut

    ref = np.asarray(DATA["fixtures"]["lut_cube_arb12"], dtype=np.uint64)
    assert np.array_equal(cube_lut(2048), ref)


@pytest.mark.parametrize("name", ["std128", "std192", "std128q"])
def test_openfhe_eval_format_matches_reference(oracle, name):
    """or_openfhe_ntt (the EVALUATION format tfhe_setup_eval ingests) equals OpenFHE's own
    SetFormat(EVALUATION) of the same coefficient-form BSK, over the whole key."""
    fx = DATA["fixtures"][f"bskeval_{name}"]
    p = refvec.params(oracle, fx["ctx"])
    bsk, _ = oracle.kat_keys(p, oracle.Rng(int(fx["keys"].split(":")[1])))
    ev = oracle.openfhe_ntt(p.Q, p.N, bsk)
    assert f"{oracle.fnv1a64(ev[:2 * p.N]):016x}" == fx["head_fnv"]
    assert f"{oracle.fnv1a64(ev):016x}" == fx["fnv"]


@pytest.mark.parametrize("name", MM_CASES)
def test_mulmatrix_model_is_the_reference(oracle, name):
    """The mm_* fixtures are outputs of the reference's own CPU function CPUGEMM (examples/GEMM.cpp:30-56,
    compiled from that file into oracle/_ref/ref_kat; GEMM.cpp:110-120 compares the GPU result against it
    bit for bit).  The harness's restatement of CiphertextMulMatrix_CUDA (cpu_boundary.cpp: the FP64 DGEMM
    + fmod of lwe-operation.cu:79-125) produced the same digest (boundary_fnv, asserted by
    tools/gen_golden.py), and refvec.mulmatrix_reference (FP64 sum, fmod, static_cast<uint64_t>)
    reproduces them bit for bit, including where they leave [0, modulus) (negative sums) or round
    (sums >= 2^53)."""
    c = refvec.case(name, DATA)
    assert c["vector"]["impl"].startswith("CPUGEMM") and c["boundary_fnv"] == c["vector"]["fnv"]
    x = refvec.inputs(c, DATA["fixtures"])
    model = refvec.mulmatrix_reference(x["in"], x["matrix"], c["args"]["modulus"])
    refvec.check(c, model.ravel(), {})
    if name == "mm_gemm":  # GEMM.cpp's config: every sum exact, so model == exact product
        small = refvec.mulmatrix_exact(x["in"][:, :4], x["matrix"][:, :3], c["args"]["modulus"])
        assert np.array_equal(small, model[:3, :4])
