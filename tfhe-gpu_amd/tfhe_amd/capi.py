"""ctypes declarations of include/tfhe_hip.h."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # tfhe-gpu_amd/
_ROOT = os.path.dirname(_PKG)
_LIB = os.environ.get("TFHE_LIB", os.path.join(_PKG, "lib", "libtfhe_hip.so"))  # override: alternative builds
HEADER = os.path.join(_ROOT, "include", "tfhe_hip.h")
ABI_VERSION = 8  # TFHE_HIP_ABI_VERSION of include/tfhe_hip.h (3: tfhe_info.replicate_*; 4: row-pointer host arrays;
                 # 5: device-resident EvalFunc / EvalFloor / EvalSign; 6: knobs.duo, info.duo_timeouts;
                 # 7: knobs.split4; 8: knobs.ks40, tfhe_rccl_selftest)

# BINFHE_PARAMSET / BINGATE (binfhe-constants.h:46-101)
PARAMSETS = {"TOY": 0, "MEDIUM": 1, "STD128_AP": 2, "STD128_APOPT": 3, "STD128": 4, "STD128_OPT": 5, "STD192": 6,
             "STD192_OPT": 7, "STD256": 8, "STD256_OPT": 9, "STD128Q": 10, "STD128Q_OPT": 11, "STD192Q": 12,
             "STD192Q_OPT": 13, "STD256Q": 14, "STD256Q_OPT": 15, "SIGNED_MOD_TEST": 16}
BINGATE = {"OR": 0, "AND": 1, "NOR": 2, "NAND": 3, "XOR_FAST": 4, "XNOR_FAST": 5, "XOR": 6, "XNOR": 7}


class TfheError(RuntimeError):
    def __init__(self, status: int, where: str, msg: str):
        super().__init__(f"{where}: status {status}: {msg}")
        self.status = status


class Params(C.Structure):
    _fields_ = [("n", C.c_uint32), ("N", C.c_uint32), ("q", C.c_uint64), ("Q", C.c_uint64), ("qKS", C.c_uint64),
                ("baseKS", C.c_uint32), ("baseG", C.c_uint32), ("numDigitsToThrow", C.c_uint32),
                ("digitsG", C.c_uint32), ("dKS", C.c_uint32), ("dG2", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}

    def bsk_words(self):
        return self.n * 2 * self.dG2 * 2 * self.N

    def ksk_words(self):
        return self.N * self.baseKS * self.dKS * (self.n + 1)


class Info(C.Structure):
    _fields_ = [("num_devices", C.c_int), ("word_bits", C.c_int), ("bsk_device_bytes", C.c_uint64),
                ("ksk_device_bytes", C.c_uint64), ("bootstraps", C.c_uint64), ("key_image_bytes", C.c_uint64),
                ("br_kernel", C.c_int), ("replicate_method", C.c_int), ("replicate_ms", C.c_double),
                ("duo_timeouts", C.c_uint32)]


class Knobs(C.Structure):
    """tfhe_knobs: launch choices of a context (include/tfhe_hip.h), environment at setup, then tfhe_set_knobs."""
    _fields_ = [(k, C.c_int32) for k in ("ks_tiled_min", "ks_cts", "ks_split", "ks_pk", "host_parts", "wire",
                                         "acc_flags", "f64w", "sf2", "generic", "trace", "probe", "duo",
                                         "sf2p", "split4", "ks40")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
VP = C.c_void_p
SZ = C.c_size_t
U64 = C.c_uint64
P = C.POINTER(Params)

_SIGS = {
    "tfhe_abi_version": ([], C.c_int),
    "tfhe_set_kernel_variant": ([C.c_int], C.c_int),
    "tfhe_get_kernel_variant": ([], C.c_int),
    "tfhe_last_error": ([], C.c_char_p),
    "tfhe_status_string": ([C.c_int], C.c_char_p),
    "tfhe_params_from_set": ([C.c_int, P], C.c_int),
    "tfhe_params_from_logq": ([C.c_int, C.c_int, C.c_uint32, C.c_int64, C.c_uint32, C.c_uint32, P], C.c_int),
    "tfhe_params_finish": ([P], C.c_int),
    "tfhe_setup": ([C.POINTER(VP), P, u64p, u64p, C.c_int], C.c_int),
    "tfhe_setup_eval": ([C.POINTER(VP), P, u64p, u64p, C.c_int], C.c_int),
    "tfhe_clean": ([VP], C.c_int),
    "tfhe_eval_acc": ([VP, SZ, u64p, U64, u64p], C.c_int),
    "tfhe_shard_range": ([SZ, C.c_int, C.c_int, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)], C.c_int),
    "tfhe_host_shard_selftest": ([SZ, C.c_int, C.c_int, C.POINTER(C.c_size_t)], C.c_int),
    "tfhe_rccl_selftest": ([C.c_int, SZ, C.c_char_p, C.POINTER(C.c_int)], C.c_int),
    "tfhe_eval_acc_tv": ([VP, SZ, u64p, U64, u64p, C.c_uint32, u64p], C.c_int),
    "tfhe_mkm_switch": ([VP, SZ, u64p, U64, u64p], C.c_int),
    "tfhe_eval_acc_tv_rows": ([VP, SZ, VP, U64, u64p, C.c_uint32, VP], C.c_int),
    "tfhe_mkm_switch_rows": ([VP, SZ, VP, VP, U64, VP, VP], C.c_int),
    "tfhe_ciphertext_mul_matrix": ([VP, SZ, u64p, SZ, i64p, U64, u64p], C.c_int),
    "tfhe_lwe_gpu_setup": ([C.c_int], C.c_int),
    "tfhe_lwe_gpu_clean": ([], C.c_int),
    "tfhe_eval_bin_gate": ([VP, C.c_int, SZ, u64p, u64p, U64, u64p], C.c_int),
    "tfhe_eval_func": ([VP, SZ, u64p, U64, u64p, C.c_int, u64p], C.c_int),
    "tfhe_eval_floor": ([VP, SZ, u64p, U64, C.c_uint32, u64p], C.c_int),
    "tfhe_eval_sign": ([VP, SZ, u64p, U64, u64p], C.c_int),
    "tfhe_eval_decomp": ([VP, SZ, u64p, U64, C.c_uint32, u64p, u64p, C.POINTER(C.c_uint32)], C.c_int),
    "tfhe_eval_bin_gate_device": ([VP, C.c_int, SZ, VP, VP, U64, VP, VP], C.c_int),
    "tfhe_eval_acc_device": ([VP, SZ, VP, U64, VP, VP], C.c_int),
    "tfhe_mkm_switch_device": ([VP, SZ, VP, U64, VP, VP], C.c_int),
    "tfhe_eval_func_device": ([VP, SZ, VP, U64, VP, C.c_int, VP, VP], C.c_int),
    "tfhe_eval_floor_device": ([VP, SZ, VP, U64, C.c_uint32, VP, VP], C.c_int),
    "tfhe_eval_sign_device": ([VP, SZ, VP, U64, VP, VP], C.c_int),
    "tfhe_export_key_image": ([VP, VP, SZ, VP], C.c_int),
    "tfhe_setup_from_key_image": ([C.POINTER(VP), P, VP, SZ, C.c_int], C.c_int),
    "tfhe_save_key_image": ([VP, C.c_char_p], C.c_int),
    "tfhe_setup_from_key_file": ([C.POINTER(VP), P, C.c_char_p, C.c_int], C.c_int),
    "tfhe_get_info": ([VP, C.POINTER(Info)], C.c_int),
    "tfhe_host_selftest": ([P], C.c_int),
    "tfhe_get_knobs": ([VP, C.POINTER(Knobs)], C.c_int),
    "tfhe_set_knobs": ([VP, C.POINTER(Knobs)], C.c_int),
}


def library_path() -> str:
    return _LIB


def build(jobs: int = 8) -> str:
    """Compile the HIP library for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", _PKG, f"-j{jobs}"], check=True)
    return _LIB


def exported_symbols() -> list[str]:
    """Function names declared in include/tfhe_hip.h."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(tfhe_[a-z0-9_]+)\s*\(", txt)))


TEST_LIB = os.path.join(_PKG, "lib", "libtfhe_hip_test.so")  # + fault-probe / timing builds (tests only)
_libs = {}


def lib(path: str | None = None):
    """The product library (or `path`, e.g. TEST_LIB), loaded once per path."""
    path = path or _LIB
    L = _libs.get(path)
    if L is None:
        if not os.path.exists(path):
            raise TfheError(-1, "load", f"{path} missing: run tfhe_amd.build() (make -C tfhe-gpu_amd)")
        # One HIP runtime per process: torch wheels bundle libamdhip64/libhsa-runtime64
        # with the same sonames as /opt/rocm's but are NEEDED under unversioned names,
        # so loading ours first would put two HSA runtimes on one GPU and torch would
        # then see no devices.  Loading torch first makes ours bind to its runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(path)
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name, None)  # an older build (TFHE_LIB A/B runs) may lack a newer entry point
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = res
        # the structs above mirror this ABI version.  A/B runs against the previous round's build
        # (tools/ab_lib.sh) may set TFHE_ABI_PREV=1 to admit ABI 6: its tfhe_knobs / tfhe_info are
        # prefixes of these, so reads and writes stay in bounds
        abi = L.tfhe_abi_version()
        if abi != ABI_VERSION and not (6 <= abi < ABI_VERSION and os.environ.get("TFHE_ABI_PREV") == "1"):
            raise TfheError(-1, "load", f"{path} has ABI {L.tfhe_abi_version()}, binding expects {ABI_VERSION}: "
                                        "rebuild (make -C tfhe-gpu_amd)")
        _libs[path] = L
    return L


def check(status: int, where: str, L=None):
    if status != 0:
        msg = (L or lib()).tfhe_last_error().decode(errors="replace")
        raise TfheError(status, where, msg)


def params_from_set(name: str) -> Params:
    p = Params()
    check(lib().tfhe_params_from_set(PARAMSETS[name], C.byref(p)), "tfhe_params_from_set")
    return p


def params_from_logq(name: str, arb_func: bool, logQ: int, N: int = 0, baseG: int = 0, throw: int = 0) -> Params:
    """GenerateBinFHEContext(set, arbFunc, logQ, N, GINX, false, baseG, numDigitsToThrow)."""
    p = Params()
    check(lib().tfhe_params_from_logq(PARAMSETS[name], int(arb_func), logQ, N, baseG, throw, C.byref(p)),
          "tfhe_params_from_logq")
    return p


def host_selftest(p: Params):
    check(lib().tfhe_host_selftest(C.byref(p)), "tfhe_host_selftest")
