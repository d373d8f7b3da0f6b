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


_GROUPS = {}


def run_batch(members, gpus=(1,), env=None):
    """One ref_dropin process for cases sharing (ctx, keys) (ref_driver batch=: one context and one key load;
    one GPUSetup per gpus value): {(case, gpus): JSON line}, and the process's stderr (the shim's timing lines)."""
    key = (refvec.case(members[0], DATA)["ctx"], refvec.case(members[0], DATA)["keys"])
    with tempfile.TemporaryDirectory() as tmp:
        lines, tags = [], []
        for g in gpus:
            for m in members:
                cm = refvec.case(m, DATA)
                assert (cm["ctx"], cm["keys"]) == key
                d = os.path.join(tmp, f"{m}_{g}")
                os.makedirs(d)
                toks = [f"op={cm['op']}", f"gpus={g}"]
                toks += [f"{k}={v}" for k, v in refvec.write_inputs(cm, DATA["fixtures"], d).items()]
                if cm["mod"] is not None:
                    toks.append(f"mod={cm['mod']}")
                toks += [f"{k}={v}" for k, v in cm["args"].items()]
                lines.append(" ".join(toks))
                tags.append((m, g))
        bf = os.path.join(tmp, "batch")
        with open(bf, "w") as f:
            f.write("\n".join(lines) + "\n")
        r = subprocess.run([DROPIN, f"ctx={key[0]}", f"keys={key[1]}", "api=vector", f"batch={bf}"],
                           capture_output=True, text=True, timeout=600, env=dict(os.environ, **(env or {})))
        assert r.returncode == 0, r.stderr[-2000:]
        outs = [json.loads(x) for x in r.stdout.strip().splitlines()]
    assert len(outs) == len(tags), r.stdout[-2000:]
    return dict(zip(tags, outs)), r.stderr


def run_group(name):
    """The case's JSON line from one ref_dropin process per (ctx, keys) group of CASES, run once per module."""
    c = refvec.case(name, DATA)
    key = (c["ctx"], c["keys"])
    if key not in _GROUPS:
        members = [m for m in CASES if (refvec.case(m, DATA)["ctx"], refvec.case(m, DATA)["keys"]) == key]
        _GROUPS[key] = run_batch(members)
    return _GROUPS[key][0][(name, 1)]


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built (make -C oracle -f Makefile.ref dropin)")
@pytest.mark.parametrize("name", CASES)
def test_reference_vector_api_on_mi355x(name):
    c = refvec.case(name, DATA)
    js = run_group(name)
    assert js["fnv"] == c["vector"]["fnv"], (name, js)
    for k in ("digits", "moduli", "out_mod"):
        if k in c["vector"]:
            assert js[k] == c["vector"][k], (name, k)


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built")
def test_shim_takes_the_test_vector_path():
    """EvalBinGate's accumulators reach the shim as sparse test vectors (tfhe_eval_acc_tv); an
    EvalAcc with dense accumulators takes the general path -- both give the reference's outputs."""
    # the STD128 group's one process ran the gates (sparse test vectors) and the EvalAcc cases (dense)
    c = refvec.case("std128_NAND", DATA)
    assert run_group("std128_NAND")["fnv"] == c["vector"]["fnv"]
    assert run_group("std128_acc_amod1024")["fnv"] == refvec.case("std128_acc_amod1024", DATA)["vector"]["fnv"]
    err = _GROUPS[(c["ctx"], c["keys"])][1]
    assert "marshal in (test vectors)" in err, err[-2000:]
    assert "EvalAcc marshal in B=" in err, err[-2000:]


@pytest.fixture(autouse=True)
def _shim_timing(monkeypatch):
    monkeypatch.setenv("TFHE_SHIM_TIMING", "1")


STUB = os.path.join(ROOT, "tests", "stub_rccl", "librccl_stub.so")


_MULTI = {}


@pytest.mark.skipif(not (os.path.exists(DROPIN) and os.path.exists(STUB)), reason="ref_dropin or the stub RCCL not built")
@pytest.mark.parametrize("gpus", [2, 3])
@pytest.mark.parametrize("name", ["std128_NAND_b9", "arb12_func_cube_b7", "c5a_std128q_sign_b7"])
def test_reference_vector_api_over_several_devices(name, gpus):
    """The reference's unchanged caller with GPUSetup(numGPUs > 1) (binfhecontext.cpp:349-360 ->
    bootstrapping.cu:725-764, 1005-1069): the shim's context spans `gpus` logical devices on this one GPU
    (TFHE_LOGICAL_DEVICES), replicated by the engine's RCCL branch against the stub librccl (a real
    communicator cannot hold one GPU twice; tests/test_gpu_rccl_stub.py), and the vector calls shard the
    batch (>= 2 ciphertexts per device) -- the outputs are the reference's own (tests/golden: 9 gates,
    7 EvalFunc, 7 EvalSign on the C5a context)."""
    c = refvec.case(name, DATA)
    assert c["B"] >= 2 * gpus  # every device gets a shard (engine.hip run_shards)
    # one process per case: GPUSetup(2), then GPUSetup(3), on 3 logical devices (numGPUs = 2 uses two of them)
    if name not in _MULTI:
        _MULTI[name] = run_batch([name], gpus=(2, 3), env={"TFHE_LOGICAL_DEVICES": "3", "TFHE_RCCL_LIB": STUB})
    outs, err = _MULTI[name]
    js = outs[(name, gpus)]
    assert js["fnv"] == c["vector"]["fnv"], (name, gpus, js)
    assert f"[shim] GPUSetup devices={gpus} replicate_method=1" in err, err[-2000:]  # TFHE_REPLICATE_RCCL
