"""GPU: the HIP engine reproduces the REFERENCE's own vector-API outputs.

tests/golden/ref_vectors.json holds outputs of the reference's unchanged OpenFHE vector code
(tools/gen_golden.py, oracle/_ref/ref_kat).  Every case runs here through the C-ABI library on
the same regenerated inputs -- all 8 gates, EvalAcc / MKMSwitch at the boundary, EvalFunc (the
reference's cube LUT, per-ciphertext LUTs), EvalFloor, and EvalSign / EvalFloor / EvalDecomp on
both BASELINE C5 contexts (STD128Q, logQ = 23; Qin = 2^23) -- with keys in coefficient form
(tfhe_setup) and, for the gate / sign cases, in OpenFHE's EVALUATION format (tfhe_setup_eval,
what the drop-in shim passes), whose digest is itself pinned to the reference.
"""
import pytest

import refvec

pytestmark = pytest.mark.gpu
DATA = refvec.load()
_cache = {}


def hip_ctx(capi, oracle, c, fmt="coefficient"):
    key = (c["ctx"], c["keys"], fmt)
    if key not in _cache:
        for k in list(_cache):  # one context at a time (STD128Q / logQ keys are GBs on the host)
            _cache.pop(k).GPUClean()
        po = refvec.params(oracle, c["ctx"])
        bsk, ksk = refvec.keys(c, po)
        if fmt == "evaluation":
            bsk = oracle.openfhe_ntt(po.Q, po.N, bsk)
        _cache[key] = capi.BinFHEContextHIP(refvec.params(capi, c["ctx"])).GPUSetup(bsk, ksk, bsk_format=fmt)
    return _cache[key]


@pytest.fixture(scope="module")
def capi():
    import tfhe_amd

    yield tfhe_amd
    for k in list(_cache):
        _cache.pop(k).GPUClean()


@pytest.mark.parametrize("name", [c["name"] for c in DATA["cases"] if c["op"] != "mulmatrix"])
def test_gpu_matches_reference_vector_api(capi, oracle, name):
    c = refvec.case(name, DATA)
    out, extra = refvec.run(c, DATA["fixtures"], refvec.HipOps(hip_ctx(capi, oracle, c)))
    refvec.check(c, out, extra)


EVAL_CASES = ["std128_NAND", "std128_XOR", "std128_acc_amod1024", "std192_NAND", "c5a_std128q_sign"]


@pytest.mark.parametrize("name", EVAL_CASES)
def test_gpu_eval_format_keys_match_reference(capi, oracle, name):
    """tfhe_setup_eval on OpenFHE-format keys (SetFormat(EVALUATION) of the same coefficient keys,
    pinned by the bskeval fixtures in test_oracle_ref_vectors.py) gives the reference's outputs."""
    c = refvec.case(name, DATA)
    out, extra = refvec.run(c, DATA["fixtures"], refvec.HipOps(hip_ctx(capi, oracle, c, "evaluation")))
    refvec.check(c, out, extra)
