"""BinFHEContextHIP: the vector BinFHEContext surface (binfhecontext.cpp:316-365)
over the C-ABI.  Ciphertexts are numpy uint64 arrays of shape [B, n+1]
(a[0..n-1], b), keys are flat coefficient-form arrays (see include/tfhe_hip.h)."""
from __future__ import annotations

import ctypes as C
import os
from contextlib import contextmanager

import numpy as np

from .capi import BINGATE, Info, Knobs, Params, check, lib


def _u64(x):
    return np.ascontiguousarray(x, dtype=np.uint64)


def _rows(x, width: int, what: str):
    """[B][width] view of a ciphertext batch (a single ciphertext becomes B = 1); the
    C-ABI takes bare pointers, so every shape is checked here before a call."""
    x = _u64(x)
    if x.ndim == 1:
        x = x[None]
    if x.ndim != 2 or x.shape[1] != width:
        raise ValueError(f"{what}: expected shape (B, {width}), got {x.shape}")
    return x


class BinFHEContextHIP:
    BETA = 128  # BinFHEContext::GetBeta, binfhecontext.h:348-350

    def __init__(self, params: Params, library: str | None = None):
        """library: another build of the C-ABI (capi.TEST_LIB: the test library with the fault probes)."""
        self.params = params
        self._h = C.c_void_p()
        self._L = lib(library)

    # -- GPUSetup / GPUClean (binfhecontext.cpp:349-365) --
    def GPUSetup(self, bsk_coeff, ksk, num_gpus: int = 1, bsk_format: str = "coefficient"):
        """bsk_format "coefficient" (tfhe_setup) or "evaluation": OpenFHE's NTT-domain
        values as KeyGen/BTKeyLoad leave them (tfhe_setup_eval, no host INTT)."""
        if bsk_format not in ("coefficient", "evaluation"):
            raise ValueError("bsk_format must be 'coefficient' or 'evaluation'")
        if self._h:
            self.GPUClean()
        p = self.params
        bsk = _u64(bsk_coeff).ravel()
        kk = _u64(ksk).ravel()
        if bsk.size != p.bsk_words() or kk.size != p.ksk_words():
            raise ValueError("key sizes do not match the parameters")
        fn = self._L.tfhe_setup if bsk_format == "coefficient" else self._L.tfhe_setup_eval
        self._check(fn(C.byref(self._h), C.byref(p), bsk, kk, num_gpus), fn.__name__)
        return self

    def _check(self, status, where):
        check(status, where, self._L)

    @classmethod
    def from_key_image(cls, params: Params, d_src: int, nbytes: int, device: int = 0, library: str | None = None):
        ctx = cls(params, library)
        ctx._check(ctx._L.tfhe_setup_from_key_image(C.byref(ctx._h), C.byref(params), C.c_void_p(d_src), nbytes, device),
                   "tfhe_setup_from_key_image")
        return ctx

    @classmethod
    def from_key_file(cls, params: Params, path: str, device: int = 0, library: str | None = None):
        """Adopt a key image saved by save_key_image (no host key conversion)."""
        ctx = cls(params, library)
        ctx._check(ctx._L.tfhe_setup_from_key_file(C.byref(ctx._h), C.byref(params), os.fsencode(path), device),
                   "tfhe_setup_from_key_file")
        return ctx

    def save_key_image(self, path: str):
        self._check(self._L.tfhe_save_key_image(self._h, os.fsencode(path)), "tfhe_save_key_image")

    def export_key_image(self, d_dst: int, nbytes: int, stream: int = 0):
        self._check(self._L.tfhe_export_key_image(self._h, C.c_void_p(d_dst), nbytes, C.c_void_p(stream)),
              "tfhe_export_key_image")

    def GPUClean(self):
        if self._h:
            self._check(self._L.tfhe_clean(self._h), "tfhe_clean")
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.GPUClean()
        except Exception:
            pass

    def info(self) -> Info:
        inf = Info()
        self._check(self._L.tfhe_get_info(self._h, C.byref(inf)), "tfhe_get_info")
        return inf

    @property
    def handle(self):
        return self._h

    # -- launch knobs (tfhe_knobs: environment at setup, then only these calls) --
    def knobs(self) -> dict:
        k = Knobs()
        self._check(self._L.tfhe_get_knobs(self._h, C.byref(k)), "tfhe_get_knobs")
        return k.as_dict()

    def set_knobs(self, **kw):
        k = Knobs()
        self._check(self._L.tfhe_get_knobs(self._h, C.byref(k)), "tfhe_get_knobs")
        for name, v in kw.items():
            if not hasattr(k, name):
                raise KeyError(f"unknown knob {name}")
            setattr(k, name, int(v))
        self._check(self._L.tfhe_set_knobs(self._h, C.byref(k)), "tfhe_set_knobs")

    @contextmanager
    def knobs_set(self, **kw):
        """Temporarily change knobs (tests, A/B runs); restored on exit."""
        old = self.knobs()
        self.set_knobs(**kw)
        try:
            yield self
        finally:
            self.set_knobs(**old)

    def GetBeta(self):
        return self.BETA

    def GetMaxPlaintextSpace(self):
        return self.params.q // self.BETA // 2

    # -- reference boundary calls --
    def EvalAcc(self, a, a_mod, acc):
        """EvalAcc_CUDA: a[B][n] mod a_mod, acc[B][2][N] -> new acc (acc0 transposed)."""
        n, N = self.params.n, self.params.N
        a = _u64(a)
        out = np.array(acc, dtype=np.uint64, copy=True, order="C")
        if a.size == 0 or a.size % n:
            raise ValueError(f"EvalAcc: a must hold B*n words (n = {n}), got {a.size}")
        B = a.size // n
        if out.size != B * 2 * N:
            raise ValueError(f"EvalAcc: acc must hold B*2*N = {B * 2 * N} words, got {out.size}")
        self._check(self._L.tfhe_eval_acc(self._h, B, a.ravel(), a_mod, out.ravel()), "tfhe_eval_acc")
        return out

    def MKMSwitch(self, ct_ext, fmod):
        ct_ext = _rows(ct_ext, self.params.N + 1, "MKMSwitch")
        B = ct_ext.shape[0]
        out = np.empty((B, self.params.n + 1), dtype=np.uint64)
        self._check(self._L.tfhe_mkm_switch(self._h, B, ct_ext.ravel(), fmod, out.ravel()), "tfhe_mkm_switch")
        return out

    def CiphertextMulMatrix(self, ct, matrix, modulus):
        ct = _rows(ct, self.params.n + 1, "CiphertextMulMatrix")
        m = np.ascontiguousarray(matrix, dtype=np.int64)
        if m.ndim != 2:
            raise ValueError("CiphertextMulMatrix: matrix must be 2-D [K][cols]")
        K, cols = m.shape
        if ct.size != K * (self.params.n + 1):  # lwe-operation.cu:66-69
            raise ValueError("The number of rows of the matrix must be equal to the number of input ciphertexts.")
        out = np.empty((cols, self.params.n + 1), dtype=np.uint64)
        self._check(self._L.tfhe_ciphertext_mul_matrix(self._h, K, ct.ravel(), cols, m.ravel(), modulus, out.ravel()),
              "tfhe_ciphertext_mul_matrix")
        return out

    # -- vector BinFHEContext surface --
    def _batch(self, ct, what="ciphertexts"):
        ct = _rows(ct, self.params.n + 1, what)
        return ct, ct.shape[0]

    def EvalBinGate(self, gate, ct1, ct2, q=None):
        ct1, B = self._batch(ct1, "EvalBinGate ct1")
        ct2, B2 = self._batch(ct2, "EvalBinGate ct2")
        if B != B2:  # binfhe-base-scheme.cpp:607
            raise ValueError(f"EvalBinGate: input ciphertexts size unmatched ({B} vs {B2})")
        g = BINGATE[gate] if isinstance(gate, str) else int(gate)
        out = np.empty((B, self.params.n + 1), dtype=np.uint64)
        self._check(self._L.tfhe_eval_bin_gate(self._h, g, B, ct1.ravel(), ct2.ravel(), q or self.params.q, out.ravel()),
              "tfhe_eval_bin_gate")
        return out

    def EvalFunc(self, ct, lut, q=None):
        ct, B = self._batch(ct, "EvalFunc")
        lut = _u64(lut)
        qq = q or self.params.q
        if not (lut.shape == (qq,) or lut.shape == (B, qq)):
            raise ValueError(f"EvalFunc: LUT must have shape ({qq},) or ({B}, {qq}), got {lut.shape}")
        out = np.empty((B, self.params.n + 1), dtype=np.uint64)
        self._check(self._L.tfhe_eval_func(self._h, B, ct.ravel(), qq, lut.ravel(), int(lut.ndim == 2),
                                   out.ravel()), "tfhe_eval_func")
        return out

    def EvalFloor(self, ct, mod, roundbits=0):
        ct, B = self._batch(ct, "EvalFloor")
        out = np.empty((B, self.params.n + 1), dtype=np.uint64)
        self._check(self._L.tfhe_eval_floor(self._h, B, ct.ravel(), mod, roundbits, out.ravel()), "tfhe_eval_floor")
        return out

    def EvalSign(self, ct, mod):
        ct, B = self._batch(ct, "EvalSign")
        out = np.empty((B, self.params.n + 1), dtype=np.uint64)
        self._check(self._L.tfhe_eval_sign(self._h, B, ct.ravel(), mod, out.ravel()), "tfhe_eval_sign")
        return out

    def EvalDecomp(self, ct, mod, max_digits=16):
        ct, B = self._batch(ct, "EvalDecomp")
        out = np.zeros((B, max_digits, self.params.n + 1), dtype=np.uint64)
        moduli = np.zeros(max_digits, dtype=np.uint64)
        nd = C.c_uint32()
        self._check(self._L.tfhe_eval_decomp(self._h, B, ct.ravel(), mod, max_digits, out.ravel(), moduli, C.byref(nd)),
              "tfhe_eval_decomp")
        d = nd.value
        return out[:, :d, :], [int(m) for m in moduli[:d]]

    # -- device-resident (pointers are integers, e.g. torch tensor.data_ptr()) --
    def EvalBinGateDevice(self, gate, B, d_ct1, d_ct2, d_out, q=None, stream=0):
        g = BINGATE[gate] if isinstance(gate, str) else int(gate)
        self._check(self._L.tfhe_eval_bin_gate_device(self._h, g, B, C.c_void_p(d_ct1), C.c_void_p(d_ct2),
                                              q or self.params.q, C.c_void_p(d_out), C.c_void_p(stream)),
              "tfhe_eval_bin_gate_device")

    def EvalFuncDevice(self, B, d_ct, d_lut, d_out, q=None, per_ct_lut=False, stream=0):
        self._check(self._L.tfhe_eval_func_device(self._h, B, C.c_void_p(d_ct), q or self.params.q, C.c_void_p(d_lut),
                                          int(per_ct_lut), C.c_void_p(d_out), C.c_void_p(stream)),
              "tfhe_eval_func_device")

    def EvalFloorDevice(self, B, d_ct, mod, d_out, roundbits=0, stream=0):
        self._check(self._L.tfhe_eval_floor_device(self._h, B, C.c_void_p(d_ct), mod, roundbits, C.c_void_p(d_out),
                                           C.c_void_p(stream)), "tfhe_eval_floor_device")

    def EvalSignDevice(self, B, d_ct, mod, d_out, stream=0):
        self._check(self._L.tfhe_eval_sign_device(self._h, B, C.c_void_p(d_ct), mod, C.c_void_p(d_out), C.c_void_p(stream)),
              "tfhe_eval_sign_device")
