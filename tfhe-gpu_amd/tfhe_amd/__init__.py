"""tfhe_amd -- Python binding of the MI355X-native batched CGGI/GINX bootstrapping engine.

The engine is the C-ABI shared library built from ``tfhe-gpu_amd/csrc`` (see
``include/tfhe_hip.h``).  This package only marshals numpy arrays through ctypes
and mirrors the vector ``BinFHEContext`` surface of the reference
(binfhecontext.cpp:316-365): ``GPUSetup``, ``EvalBinGate``, ``EvalFunc``,
``EvalFloor``, ``EvalSign``, ``EvalDecomp``, plus the low-level
``EvalAcc``/``MKMSwitch`` boundary calls.  There is no CPU fallback: if the
library or a GPU is missing, calls raise.
"""
from .capi import (BINGATE, PARAMSETS, TfheError, Params, lib, library_path, build, exported_symbols,
                   params_from_set, params_from_logq, host_selftest)
from .context import BinFHEContextHIP

__all__ = ["BINGATE", "PARAMSETS", "TfheError", "Params", "lib", "library_path", "build", "exported_symbols",
           "params_from_set", "params_from_logq", "host_selftest", "BinFHEContextHIP"]
