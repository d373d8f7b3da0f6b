"""GPU: the drop-in.  The reference's own, unchanged OpenFHE BinFHE code (libopenfhe_ref.so,
compiled from /root/reference by oracle/Makefile.ref) linked with the HIP shim
(tfhe-gpu_amd/shim/bootstrapping_hip.cpp) and libtfhe_hip.so -- oracle/_ref/ref_dropin -- runs
the vector API (BinFHEContext::GPUSetup / EvalBinGate / EvalFunc / EvalFloor / EvalSign /
EvalDecomp, binfhecontext.cpp:316-365) on the MI355X and must reproduce the outputs the same
code produced with the reference's CPU functions behind the seven symbols
(tests/golden/ref_vectors.json).  The binary is built in the development container (it needs
the reference's sources) and travels with the tree; without it the test is skipped.
"""
import json
import os
import subprocess
import tempfile

import pytest

import refvec

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ref_dropin")
DATA = refvec.load()
CASES = ["std128_NAND", "std128_AND", "std128_XOR", "std128_XNOR_FAST", "std128_acc_amod1024", "std128_acc_amod512",
         "std128_mkm_fmod2048", "std192_NAND", "arb12_func_cube", "arb12_funcvec", "arb12_floor",
         "c5a_std128q_sign", "c5a_std128q_decomp", "c5b_sign23_sign", "c5b_sign23_floor", "toy4096_funcvec",
         "toy8192_sign"]


def run_dropin(c, tmp, extra=()):
    files = refvec.write_inputs(c, DATA["fixtures"], tmp)
    args = [DROPIN, f"ctx={c['ctx']}", f"keys={c['keys']}", f"op={c['op']}", "api=vector", "gpus=1"]
    args += [f"{k}={v}" for k, v in files.items()]
    if c["mod"] is not None:
        args.append(f"mod={c['mod']}")
    args += [f"{k}={v}" for k, v in c["args"].items()] + list(extra)
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built (make -C oracle -f Makefile.ref dropin)")
@pytest.mark.parametrize("name", CASES)
def test_reference_vector_api_on_mi355x(name):
    c = refvec.case(name, DATA)
    with tempfile.TemporaryDirectory() as tmp:
        js, _ = run_dropin(c, tmp)
    assert js["fnv"] == c["vector"]["fnv"], (name, js)
    for k in ("digits", "moduli", "out_mod"):
        if k in c["vector"]:
            assert js[k] == c["vector"][k], (name, k)


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built")
def test_shim_takes_the_test_vector_path():
    """EvalBinGate's accumulators reach the shim as sparse test vectors (tfhe_eval_acc_tv); an
    EvalAcc with dense accumulators takes the general path -- both give the reference's outputs."""
    with tempfile.TemporaryDirectory() as tmp:
        _, err = run_dropin(refvec.case("std128_NAND", DATA), tmp)
        assert "marshal in (test vectors)" in err, err[-2000:]
        _, err = run_dropin(refvec.case("std128_acc_amod1024", DATA), tmp)
        assert "EvalAcc marshal in B=" in err, err[-2000:]


@pytest.fixture(autouse=True)
def _shim_timing(monkeypatch):
    monkeypatch.setenv("TFHE_SHIM_TIMING", "1")
