#!/usr/bin/env python3
"""Throughput of the other SURVEY.md 8(d) configurations on one MI355X (C3, C4, C5a, C5b; F11 /
F11t0: EvalFloor in the reference example's logQ = 11 context, with / without the thrown digit).

bench.py measures the headline C2 (STD128 NAND, inputs resident in HBM).  This script
times the host-array entry points (EvalFunc / EvalBinGate / EvalSign: PCIe transfers
included) with synthetic keys (the SURVEY Appendix B splitmix64 recipe, bench.synthetic_keys) and
random ciphertexts, counting bootstraps with the engine's own counter (tfhe_info.bootstraps).  C3's
LUT is the reference's GenerateLUTviaFunction(x^3 mod 8) (tests/helpers.cube_lut, pinned to the
reference's own LUT by tests/test_oracle_ref_vectors.py).  Every timed configuration is gated on
parity: the first --check ciphertexts of the timed call are recomputed by the C oracle (oracle/,
pinned to the reference) with the same keys and must be bit-identical ("parity" in the line; the
script exits non-zero otherwise).  One JSON line per configuration.
Usage: python3 tools/bench_configs.py [C3 C4 C5a C5b] [--reps 2] [--check 4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-gpu_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["C3", "C4", "C5a", "C5b"])
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--check", type=int, default=4, help="ciphertexts compared with the oracle (0: no gate)")
    args = ap.parse_args()
    import tfhe_amd
    from tfhe_amd import capi
    from bench import synthetic_keys
    from helpers import cube_lut
    failed = []

    for name in args.configs:
        if name == "C2host":  # the headline workload through the host-array API (PCIe included)
            p = capi.params_from_set("STD128")
            B, op = 8192, "EvalBinGate(NAND)"
        elif name == "C3":      # STD128 arbFunc logQ=12 throw=1, EvalFunc with an arbitrary LUT, B=4096
            p = capi.params_from_logq("STD128", True, 12, 0, 0, 1)
            B, op = 4096, "EvalFunc(x^3 mod 8)"
        elif name == "C4":    # STD192 NAND (8192 per GPU of the 65536-gate, 8-GPU config)
            p = capi.params_from_set("STD192")
            B, op = 8192, "EvalBinGate(NAND)"
        elif name == "C5a":   # STD128Q EvalSign, ciphertext modulus 2^23, B=1024
            p = capi.params_from_set("STD128Q")
            B, op = 1024, "EvalSign(Qin=2^23)"
        elif name in ("F11", "F11t0"):  # EvalFloor in the logQ = 11 context (time-estimate.cpp:100), B=4096
            p = capi.params_from_logq("STD128", False, 11, 0, 0, 1 if name == "F11" else 0)
            B, op = 4096, "EvalFloor(roundbits=1)"
        elif name == "C5b":   # STD128 logQ=23 throw=1 EvalSign, ciphertext modulus 2^23, B=1024
            p = capi.params_from_logq("STD128", False, 23, 0, 0, 1)
            B, op = 1024, "EvalSign(Qin=2^23)"
        else:
            raise SystemExit(f"unknown config {name}")
        rs = np.random.default_rng(1)
        t0 = time.perf_counter()
        bsk, ksk = synthetic_keys(p)
        ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
        setup_s = time.perf_counter() - t0
        qin = 1 << 23
        if name == "C3":
            ct = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
            lut = cube_lut(p.q)
            call = lambda: ctx.EvalFunc(ct, lut)
            ref = lambda o, k: o.eval_func(ct[:k], lut)
        elif name in ("F11", "F11t0"):
            ct = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
            call = lambda: ctx.EvalFloor(ct, p.q, 1)
            ref = lambda o, k: o.eval_floor(ct[:k], p.q, 1)
        elif name in ("C4", "C2host"):
            c1 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
            c2 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
            call = lambda: ctx.EvalBinGate("NAND", c1, c2)
            ref = lambda o, k: o.eval_bin_gate("NAND", c1[:k], c2[:k])
        else:
            ct = rs.integers(0, qin, (B, p.n + 1), dtype=np.uint64)
            call = lambda: ctx.EvalSign(ct, qin)
            ref = lambda o, k: o.eval_sign(ct[:k], qin)
        call()  # warm-up
        b0 = ctx.info().bootstraps
        t0 = time.perf_counter()
        for _ in range(args.reps):
            out = call()
        dt = time.perf_counter() - t0
        parity = None
        if args.check:
            import pyoracle

            po = (pyoracle.params_from_set({"C2host": "STD128", "C4": "STD192", "C5a": "STD128Q"}[name])
                  if name in ("C2host", "C4", "C5a") else
                  pyoracle.params_from_logq("STD128", name == "C3", {"C3": 12, "C5b": 23}.get(name, 11), 0, 0,
                                            0 if name == "F11t0" else 1))
            orc = pyoracle.Oracle(po, bsk, ksk)
            k = min(args.check, B)
            parity = {"checked": k, "bit_exact": bool(np.array_equal(out[:k], ref(orc, k))),
                      "vs": "oracle/tfhe_oracle.c, same keys and inputs"}
            orc.close()
            if not parity["bit_exact"]:
                failed.append(name)
        del bsk, ksk
        nb = ctx.info().bootstraps - b0
        info = ctx.info()
        print(json.dumps({
            "config": name, "op": op, "batch": B, "params": {"n": p.n, "N": p.N, "Q": p.Q, "dG2": p.dG2,
                                                              "baseG": p.baseG, "qKS": p.qKS},
            "kernel": ["generic", "fast", "f64", "f64-fold", "rns", "sf"][info.br_kernel],
            "bootstraps_per_call": nb // args.reps, "bootstraps_per_s": round(nb / dt, 1),
            "calls_per_s": round(args.reps / dt, 3), "note": "host-array API, PCIe transfers included",
            "setup_s": round(setup_s, 1), "parity": parity}), flush=True)
        ctx.GPUClean()
    if failed:
        raise SystemExit(f"parity FAILED: {failed}")


if __name__ == "__main__":
    main()
