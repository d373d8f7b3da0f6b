"""Shared test helpers: KAT input regeneration (SURVEY.md Appendix B recipe),
LUT construction, random ciphertext batches."""
import numpy as np


def kat_params(po, name):
    if name == "std128":
        return po.params_from_set("STD128")
    if name == "std192":
        return po.params_from_set("STD192")
    if name == "arb12":
        return po.params_from_logq("STD128", True, 12, 0, 0, 1)
    raise KeyError(name)


def kat_inputs(po, name):
    """Regenerate the KAT keys and 3 trials (a1,b1,a2,b2 each) from splitmix64 seed 1."""
    p = kat_params(po, name)
    rng = po.Rng(1)
    bsk, ksk = po.kat_keys(p, rng)
    trials = []
    for _ in range(3):
        a1 = po.splitmix(rng, p.n, p.q)
        b1 = po.splitmix(rng, 1, p.q)
        a2 = po.splitmix(rng, p.n, p.q)
        b2 = po.splitmix(rng, 1, p.q)
        trials.append((np.concatenate([a1, b1]), np.concatenate([a2, b2])))
    return p, bsk, ksk, trials


def cube_lut(q, P=8):
    """GenerateLUTviaFunction(m^3 mod p, p) (binfhecontext.cpp:280-301; time-estimate.cpp:70-75)."""
    interval = q // P

    def f(m, p1):
        return (m * m * m) % p1 if m < p1 else ((m - p1 // 2) ** 3) % p1

    return np.array([f(i // interval, P) * interval for i in range(q)], dtype=np.uint64)


def random_cts(rs, B, n, mod):
    return rs.integers(0, mod, (B, n + 1), dtype=np.uint64)
