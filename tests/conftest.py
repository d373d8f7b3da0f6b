import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "tfhe-gpu_amd", "tests"):
    path = os.path.join(ROOT, sub)
    if path not in sys.path:
        sys.path.insert(0, path)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: CPU test taking more than ~10 s")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.build()
    return pyoracle


# Contexts shared by the GPU modules (session scope): the logQ contexts' keys are 4.8 GB of KSK, and building one
# (keys, device setup, the oracle's copy) costs 4-8 s, so modules that only need *some* valid-shape keys for a
# context take them from here instead of building their own.  Keys: Appendix B splitmix64 keys, seed 97.
# shared_kat(name) -> dict(op, cp, ctx, orc); shared_kat(name, test_lib=True) sets the context up on the test
# library (the probe builds).  Product-library contexts must end the session with no duo timeouts.
SHARED_SPECS = {
    "STD128": ("set", "STD128"),
    "STD128Q": ("set", "STD128Q"),
    "STD192": ("set", "STD192"),
    "ARB12": ("logq", "STD128", True, 12, 0, 0, 1),       # C3: one transformed digit
    "LOGQ23": ("logq", "STD128", False, 23, 0, 0, 1),     # C5b: two
    "CHES18": ("logq", "STD128", True, 12, 0, 1 << 18, 0),  # CHES-experiments EvalFunc: three
}


def shared_params(module, name):
    spec = SHARED_SPECS[name]
    return module.params_from_set(spec[1]) if spec[0] == "set" else module.params_from_logq(*spec[1:])


@pytest.fixture(scope="session")
def shared_kat(oracle):
    cache = {}

    def get(name, test_lib=False):
        key = (name, test_lib)
        if key not in cache:
            import tfhe_amd

            op, cp = shared_params(oracle, name), shared_params(tfhe_amd, name)
            bsk, ksk = oracle.kat_keys(op, oracle.Rng(97))
            lib = tfhe_amd.capi.TEST_LIB if test_lib else None
            ctx = tfhe_amd.BinFHEContextHIP(cp, library=lib).GPUSetup(bsk, ksk)
            orc = oracle.Oracle(op, bsk, ksk)
            del bsk, ksk
            cache[key] = dict(op=op, cp=cp, ctx=ctx, orc=orc)
        return cache[key]

    yield get
    timeouts = {k[0]: v["ctx"].info().duo_timeouts for k, v in cache.items() if not k[1]}
    for v in cache.values():
        v["ctx"].GPUClean()
        v["orc"].close()
    assert not any(timeouts.values()), timeouts
