"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  See
tfhe_oracle.h for the reference lines each entry point restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")


class Params(C.Structure):
    _fields_ = [
        ("n", C.c_uint32), ("N", C.c_uint32), ("q", C.c_uint64), ("Q", C.c_uint64), ("qKS", C.c_uint64),
        ("baseKS", C.c_uint32), ("baseG", C.c_uint32), ("numDigitsToThrow", C.c_uint32),
        ("digitsG", C.c_uint32), ("dKS", C.c_uint32), ("dG2", C.c_uint32), ("logG", C.c_uint32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Rng(C.Structure):
    _fields_ = [("s", C.c_uint64)]


# BINFHE_PARAMSET / BINGATE numbering (binfhe-constants.h:46-101)
SETS = {"TOY": 0, "MEDIUM": 1, "STD128_AP": 2, "STD128_APOPT": 3, "STD128": 4, "STD128_OPT": 5, "STD192": 6,
        "STD192_OPT": 7, "STD256": 8, "STD256_OPT": 9, "STD128Q": 10, "STD128Q_OPT": 11, "STD192Q": 12,
        "STD192Q_OPT": 13, "STD256Q": 14, "STD256Q_OPT": 15, "SIGNED_MOD_TEST": 16}
GATES = {"OR": 0, "AND": 1, "NOR": 2, "NAND": 3, "XOR_FAST": 4, "XNOR_FAST": 5, "XOR": 6, "XNOR": 7}


def build():
    """Compile liboracle.so in place (gcc, OpenMP)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER(Params)
        L.or_params_from_set.argtypes = [C.c_int, P]
        L.or_params_from_logq.argtypes = [C.c_int, C.c_int, C.c_uint32, C.c_int64, C.c_uint32, C.c_uint32, P]
        L.or_roundqQ.argtypes = [C.c_uint64] * 3
        L.or_roundqQ.restype = C.c_uint64
        L.or_is_prime.argtypes = [C.c_uint64]
        L.or_polymul_schoolbook.argtypes = [P, u64p, u64p, u64p]
        L.or_polymul_ntt.argtypes = [P, u64p, u64p, u64p]
        L.or_signed_digit_decompose.argtypes = [P, u64p, u64p]
        L.or_create.argtypes = [P, u64p, u64p]
        L.or_create.restype = C.c_void_p
        L.or_destroy.argtypes = [C.c_void_p]
        L.or_set_threads.argtypes = [C.c_int]
        L.or_splitmix64.argtypes = [C.POINTER(Rng)]
        L.or_splitmix64.restype = C.c_uint64
        L.or_splitmix_fill.argtypes = [C.POINTER(Rng), C.c_size_t, C.c_uint64, u64p]
        L.or_fnv1a64.argtypes = [u64p, C.c_size_t]
        L.or_fnv1a64.restype = C.c_uint64
        L.or_kat_keys.argtypes = [P, C.POINTER(Rng), u64p, u64p]
        L.or_root_of_unity.argtypes = [C.c_uint64, C.c_uint32]
        L.or_root_of_unity.restype = C.c_uint64
        L.or_openfhe_ntt.argtypes = [C.c_uint64, C.c_uint32, C.c_size_t, u64p, u64p, C.c_int]
        L.or_keygen.argtypes = [P, C.POINTER(Rng), u64p, u64p, u64p]
        L.or_encrypt.argtypes = [P, C.POINTER(Rng), u64p, C.c_int64, C.c_uint64, C.c_uint64, u64p]
        L.or_decrypt.argtypes = [P, u64p, u64p, C.c_uint64, C.c_uint64]
        L.or_decrypt.restype = C.c_int64
        L.or_eval_acc.argtypes = [C.c_void_p, C.c_size_t, u64p, C.c_uint64, u64p]
        L.or_mkm_switch.argtypes = [C.c_void_p, C.c_size_t, u64p, C.c_uint64, u64p]
        L.or_eval_bin_gate.argtypes = [C.c_void_p, C.c_int, C.c_size_t, u64p, u64p, C.c_uint64, u64p]
        L.or_eval_func.argtypes = [C.c_void_p, C.c_size_t, u64p, C.c_uint64, u64p, u64p]
        L.or_eval_func_vec.argtypes = [C.c_void_p, C.c_size_t, u64p, C.c_uint64, u64p, u64p]
        L.or_eval_floor.argtypes = [C.c_void_p, C.c_size_t, u64p, C.c_uint64, C.c_uint32, u64p]
        L.or_eval_sign.argtypes = [C.c_void_p, C.c_size_t, u64p, C.c_uint64, u64p]
        L.or_eval_decomp.argtypes = [C.c_void_p, C.c_size_t, u64p, C.c_uint64, C.c_uint32, u64p, u64p]
        L.or_bootstrap_count.argtypes = [C.c_void_p]
        L.or_bootstrap_count.restype = C.c_uint64
        _lib = L
    return _lib


def params_from_set(name: str) -> Params:
    p = Params()
    rc = lib().or_params_from_set(SETS[name], C.byref(p))
    if rc != 0:
        raise ValueError(f"unknown parameter set {name}")
    return p


def params_from_logq(name: str, arb_func: bool, logQ: int, N: int = 0, baseG: int = 0, throw: int = 0) -> Params:
    p = Params()
    rc = lib().or_params_from_logq(SETS[name], int(arb_func), logQ, N, baseG, throw, C.byref(p))
    if rc != 0:
        raise ValueError(f"invalid logQ parameter request (rc={rc})")
    return p


def sizes(p: Params):
    nb = p.n * 2 * p.dG2 * 2 * p.N
    nk = p.N * p.baseKS * p.dKS * (p.n + 1)
    return nb, nk


def kat_keys(p: Params, rng: Rng):
    nb, nk = sizes(p)
    bsk = np.empty(nb, dtype=np.uint64)
    ksk = np.empty(nk, dtype=np.uint64)
    lib().or_kat_keys(C.byref(p), C.byref(rng), bsk, ksk)
    return bsk, ksk


def keygen(p: Params, rng: Rng):
    nb, nk = sizes(p)
    sk = np.empty(p.n, dtype=np.uint64)
    bsk = np.empty(nb, dtype=np.uint64)
    ksk = np.empty(nk, dtype=np.uint64)
    lib().or_keygen(C.byref(p), C.byref(rng), sk, bsk, ksk)
    return sk, bsk, ksk


def root_of_unity(Q: int, N: int) -> int:
    """RootOfUnity(2N, Q): the smallest primitive 2N-th root (nbtheory.cpp:284-343)."""
    return int(lib().or_root_of_unity(Q, N))


def openfhe_ntt(Q: int, N: int, polys, inverse: bool = False) -> np.ndarray:
    """COEFFICIENT <-> OpenFHE EVALUATION format of a stack of N-word polynomials."""
    a = np.ascontiguousarray(polys, dtype=np.uint64).ravel()
    out = np.empty_like(a)
    lib().or_openfhe_ntt(Q, N, a.size // N, a, out, int(inverse))
    return out


def splitmix(rng: Rng, count: int, mod: int) -> np.ndarray:
    out = np.empty(count, dtype=np.uint64)
    lib().or_splitmix_fill(C.byref(rng), count, mod, out)
    return out


def encrypt(p: Params, rng: Rng, sk, m: int, ptxt_mod: int, mod: int) -> np.ndarray:
    ct = np.empty(p.n + 1, dtype=np.uint64)
    lib().or_encrypt(C.byref(p), C.byref(rng), sk, m, ptxt_mod, mod, ct)
    return ct


def decrypt(p: Params, sk, ct, ptxt_mod: int, mod: int) -> int:
    return int(lib().or_decrypt(C.byref(p), sk, np.ascontiguousarray(ct, dtype=np.uint64), ptxt_mod, mod))


def fnv1a64(values) -> int:
    if isinstance(values, np.ndarray) and values.dtype == np.uint64:
        return int(lib().or_fnv1a64(np.ascontiguousarray(values).ravel(), values.size))
    h = 0xCBF29CE484222325
    for v in values:
        v = int(v)
        for i in range(8):
            h ^= (v >> (8 * i)) & 0xFF
            h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


class Oracle:
    """An oracle context owning its keys (or_ctx)."""

    def __init__(self, p: Params, bsk, ksk, threads: int = 0):
        self.p = p
        self.L = lib()
        if threads:
            self.L.or_set_threads(threads)
        self.h = self.L.or_create(C.byref(p), np.ascontiguousarray(bsk, dtype=np.uint64),
                                  np.ascontiguousarray(ksk, dtype=np.uint64))

    def close(self):
        if self.h:
            self.L.or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def bootstraps(self) -> int:
        return int(self.L.or_bootstrap_count(self.h))

    def eval_acc(self, a, amod, acc):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        acc = np.array(acc, dtype=np.uint64, copy=True, order="C")
        B = a.size // self.p.n
        self.L.or_eval_acc(self.h, B, a.ravel(), amod, acc.ravel())
        return acc

    def mkm_switch(self, ct_ext, fmod):
        ct_ext = np.ascontiguousarray(ct_ext, dtype=np.uint64)
        B = ct_ext.size // (self.p.N + 1)
        out = np.empty((B, self.p.n + 1), dtype=np.uint64)
        self.L.or_mkm_switch(self.h, B, ct_ext.ravel(), fmod, out.ravel())
        return out

    def _b(self, ct):
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        return ct, ct.size // (self.p.n + 1)

    def eval_bin_gate(self, gate, ct1, ct2, q=None):
        ct1, B = self._b(ct1)
        ct2, _ = self._b(ct2)
        out = np.empty((B, self.p.n + 1), dtype=np.uint64)
        g = GATES[gate] if isinstance(gate, str) else int(gate)
        rc = self.L.or_eval_bin_gate(self.h, g, B, ct1.ravel(), ct2.ravel(), q or self.p.q, out.ravel())
        if rc != 0:
            raise RuntimeError(f"or_eval_bin_gate rc={rc}")
        return out

    def eval_func(self, ct, lut, q=None):
        ct, B = self._b(ct)
        out = np.empty((B, self.p.n + 1), dtype=np.uint64)
        lut = np.ascontiguousarray(lut, dtype=np.uint64)
        q = q or self.p.q
        fn = self.L.or_eval_func_vec if lut.ndim == 2 else self.L.or_eval_func
        rc = fn(self.h, B, ct.ravel(), q, lut.ravel(), out.ravel())
        if rc != 0:
            raise RuntimeError(f"or_eval_func rc={rc}")
        return out

    def eval_floor(self, ct, mod, roundbits=0):
        ct, B = self._b(ct)
        out = np.empty((B, self.p.n + 1), dtype=np.uint64)
        rc = self.L.or_eval_floor(self.h, B, ct.ravel(), mod, roundbits, out.ravel())
        if rc != 0:
            raise RuntimeError(f"or_eval_floor rc={rc}")
        return out

    def eval_sign(self, ct, mod):
        ct, B = self._b(ct)
        out = np.empty((B, self.p.n + 1), dtype=np.uint64)
        rc = self.L.or_eval_sign(self.h, B, ct.ravel(), mod, out.ravel())
        if rc != 0:
            raise RuntimeError(f"or_eval_sign rc={rc}")
        return out

    def eval_decomp(self, ct, mod, max_digits=16):
        ct, B = self._b(ct)
        out = np.zeros((B, max_digits, self.p.n + 1), dtype=np.uint64)
        moduli = np.zeros(max_digits, dtype=np.uint64)
        d = self.L.or_eval_decomp(self.h, B, ct.ravel(), mod, max_digits, out.ravel(), moduli)
        if d < 0:
            raise RuntimeError(f"or_eval_decomp rc={d}")
        return out[:, :d, :], [int(m) for m in moduli[:d]]
