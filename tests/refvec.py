"""Inputs of the reference-generated golden vectors (tests/golden/ref_vectors.json).

Every input array of a case is regenerated here from its spec -- splitmix64(seed) values
mod `mod` (pyoracle.splitmix, the SURVEY Appendix B generator), reshaped to `shape` -- or
taken from a fixture in the same file ({"golden": name}).  tools/gen_golden.py wrote the
outputs by running the reference on exactly these arrays.
"""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_vectors.json")


def ct_spec(seed, B, n, mod):
    return {"seed": seed, "shape": [B, n + 1], "mod": mod}


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def case(name, data=None):
    data = data or load()
    for c in data["cases"]:
        if c["name"] == name:
            return c
    raise KeyError(name)


def gen(spec, fixtures):
    import pyoracle

    if "golden" in spec:
        return np.asarray(fixtures[spec["golden"]], dtype=np.uint64)
    shape = spec["shape"]
    count = int(np.prod(shape))
    v = pyoracle.splitmix(pyoracle.Rng(spec["seed"]), count, spec["mod"]).reshape(shape)
    if "offset" in spec:  # signed entries (CiphertextMulMatrix's int64 matrix): value - offset
        v = v.astype(np.int64) - np.int64(spec["offset"])
    if "scale" in spec:   # large entries: value * scale (int64)
        v = v.astype(np.int64) * np.int64(spec["scale"])
    return v


def inputs(c, fixtures):
    return {k: gen(v, fixtures) for k, v in c["inputs"].items()}


def write_inputs(c, fixtures, tmpdir):
    files = {}
    for k, arr in inputs(c, fixtures).items():
        path = os.path.join(tmpdir, f"{k}.bin")
        arr = np.ascontiguousarray(arr)
        (arr.view(np.uint64) if arr.dtype == np.int64 else arr.astype(np.uint64)).tofile(path)
        files[k] = path
    return files


def params(module, ctx):
    """ctx spec of ref_driver ("set:NAME" / "logq:SET,arb,logQ,N,baseG,throw") -> module's Params
    (pyoracle or tfhe_amd, which expose the same two constructors)."""
    kind, spec = ctx.split(":", 1)
    if kind == "set":
        return module.params_from_set(spec)
    s, arb, logq, N, baseG, thr = spec.split(",")
    return module.params_from_logq(s, bool(int(arb)), int(logq), int(N), int(baseG), int(thr))


def keys(c, p_oracle):
    """keys=synth:<seed>: the Appendix B splitmix64 coefficient-form keys (ref_driver load_keys)."""
    import pyoracle

    kind, seed = c["keys"].split(":")
    assert kind == "synth", c["keys"]
    return pyoracle.kat_keys(p_oracle, pyoracle.Rng(int(seed)))


class OracleOps:
    def __init__(self, o):
        self.o = o

    def acc(self, a, amod, acc):
        return self.o.eval_acc(a, amod, acc)

    def mkm(self, ext, fmod):
        return self.o.mkm_switch(ext, fmod)

    def gate(self, g, c1, c2, q):
        return self.o.eval_bin_gate(g, c1, c2, q)

    def func(self, ct, lut, q):
        return self.o.eval_func(ct, lut, q)

    def floor(self, ct, mod, rb):
        return self.o.eval_floor(ct, mod, rb)

    def sign(self, ct, mod):
        return self.o.eval_sign(ct, mod)

    def decomp(self, ct, mod):
        return self.o.eval_decomp(ct, mod)


class HipOps:
    def __init__(self, ctx):
        self.c = ctx

    def acc(self, a, amod, acc):
        return self.c.EvalAcc(a, amod, acc)

    def mkm(self, ext, fmod):
        return self.c.MKMSwitch(ext, fmod)

    def gate(self, g, c1, c2, q):
        return self.c.EvalBinGate(g, c1, c2, q)

    def func(self, ct, lut, q):
        return self.c.EvalFunc(ct, lut, q)

    def floor(self, ct, mod, rb):
        return self.c.EvalFloor(ct, mod, rb)

    def sign(self, ct, mod):
        return self.c.EvalSign(ct, mod)

    def decomp(self, ct, mod):
        return self.c.EvalDecomp(ct, mod)


def run(c, fixtures, ops):
    """Runs case c on `ops`; returns (flat u64 output in ref_driver's layout, extra dict)."""
    x = inputs(c, fixtures)
    op, mod = c["op"], c["mod"]
    extra = {}
    if op == "acc":
        out = ops.acc(x["in"], mod, x["acc"])
    elif op == "mkm":
        out = ops.mkm(x["in"], c["args"]["fmod"])
    elif op in ("func", "funcvec"):
        out = ops.func(x["in"], x["lut"], mod)
    elif op == "floor":
        out = ops.floor(x["in"], mod, int(c["args"].get("roundbits", 0)))
    elif op == "sign":
        out = ops.sign(x["in"], mod)
    elif op == "decomp":
        out, moduli = ops.decomp(x["in"], mod)
        extra = {"moduli": moduli, "digits": len(moduli)}
    else:
        out = ops.gate(op, x["in"], x["in2"], mod)
    return np.ascontiguousarray(out, dtype=np.uint64).ravel(), extra


def check(c, out, extra):
    """Asserts that `out` is the reference's vector output of case c."""
    import pyoracle

    want = c["vector"]
    assert out.size == want["words"], (c["name"], out.size, want["words"])
    assert [int(v) for v in out[:4]] == want["head"], (c["name"], out[:4], want["head"])
    assert int(out[-1]) == want["last"], c["name"]
    assert f"{pyoracle.fnv1a64(out):016x}" == want["fnv"], c["name"]
    for k in ("moduli", "digits"):
        if k in want:
            assert extra[k] == want[k], (c["name"], k, extra[k], want[k])


def mulmatrix_reference(ct, mat, modulus):
    """CiphertextMulMatrix as the reference computes it (lwe-operation.cu:79-125): ciphertext words and
    matrix entries as doubles, out[c] = sum_k mat[k][c] ct[k] in FP64 (k = 0 .. K-1 in order: cuBLAS's
    order is unspecified, every sum below 2^53 is exact in any order), fmod(., modulus), then
    static_cast<uint64_t> -- a negative fmod result wraps as x86-64 converts it (cvttsd2si): 2^64 - |r|.
    Returns [cols][n+1] u64."""
    A = np.asarray(ct, dtype=np.uint64).astype(np.float64)          # [K][n+1]
    W = np.asarray(mat, dtype=np.int64).astype(np.float64)          # [K][cols]
    C = np.zeros((W.shape[1], A.shape[1]), dtype=np.float64)
    for k in range(A.shape[0]):
        C += W[k][:, None] * A[k][None, :]
    return np.fmod(C, float(modulus)).astype(np.int64).view(np.uint64)


def mulmatrix_exact(ct, mat, modulus):
    """The exact product sum_k mat[k][c] ct[k] mod modulus in [0, modulus) (the HIP kernel's definition)."""
    A = [[int(x) for x in row] for row in np.asarray(ct, dtype=np.uint64)]
    W = np.asarray(mat, dtype=np.int64)
    out = np.empty((W.shape[1], len(A[0])), dtype=np.uint64)
    for c in range(W.shape[1]):
        col = [int(w) for w in W[:, c]]
        for j in range(len(A[0])):
            out[c, j] = sum(col[k] * A[k][j] for k in range(len(A))) % modulus
    return out
