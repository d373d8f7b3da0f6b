#!/usr/bin/env python3
"""bench.py -- bootstraps/sec of the batched GINX bootstrap on MI355X.

Default workload (BASELINE.json configs[1], "C2"): STD128 (n=512, N=1024, Q=2^27-2^11+1,
baseG=2^7) EvalBinGate(NAND), batch 8192 per GPU.  One step = one vector EvalBinGate call
over the batch with both input vectors already resident in HBM: test vector -> blind
rotation (n external products) -> extraction -> MKM, all on device (the fused
tfhe_eval_bin_gate_device entry point).  One bootstrap per gate.

--config selects the other SURVEY.md 8(d) configurations, measured the same way (device-resident
step, the dominant kernel timed alone, the matching VALU peak, PMC from a per-config record, the
reference's CPU path on the same context, keys and inputs):
  C3   STD128 arbFunc logQ=12 throw=1, EvalFunc(x^3 mod 8) (arbitrary LUT: 2 bootstraps), 4096 per GPU
  C4   STD192 EvalBinGate(NAND), 8192 per GPU (65536 on 8 GPUs)
  C5a  STD128Q EvalSign, ciphertext modulus 2^23 (15 bootstraps each), 1024 in all (strong scaling)
  C5b  STD128 logQ=23 throw=1 EvalSign, modulus 2^23 (7 bootstraps each), 1024 in all (strong scaling)

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process
per GPU; the key image is built once on rank 0 and broadcast over RCCL/xGMI (torch.distributed,
backend "nccl" = RCCL), then every rank bootstraps its own shard with no data-path collective.
WORLD_SIZE must equal --gpus (exit status 2 otherwise).

Extra JSON fields:
  dist          backend and world size torch.distributed reports, per-rank blind-rotation kernel
                times (max / min), the key broadcast time.
  roofline      the blind-rotation kernel (the dominant one), timed alone with HIP events on its
                stream.  Its bound is integer VALU issue: bound "valu-int",
                achieved = the algorithmic modular multiplies of SURVEY 8(d) (n[(dG2+2)(N/2)log2 N +
                4 dG2 N + 4N] per bootstrap) per second, peak = the microbenchmarked rate of the
                product that kernel issues (tools/microbench/valu_rates.hip, --valu-peak-json:
                signed Montgomery for STD128, exact FP64 fmodmul at the context's Q for STD192 /
                STD128Q, special-form u64 for the 54-bit Q), frac = their ratio.  traffic = PMC HBM
                bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md
                corrections; --pmc-json), hbm_frac = traffic / kernel time / 8 TB/s,
                effective_keystream_tbs = SURVEY B_alg (BSK + KS gather + LWE I/O per bootstrap, no
                cross-ciphertext reuse) x batch / kernel time.
  valu          PMC view of the same kernel: VALU instructions, busy fraction, the clock the part
                held under it.
  value_end_to_end / host_array  the same op through the host-array entry point (PCIe copies,
                pinned staging and the host thread included), same inputs, whole job.
  dropin        (C2) the reference's own, unchanged vector EvalBinGate (OpenFHE BinFHE code
                compiled from its sources, oracle/_ref/ref_dropin) running on this GPU through the
                drop-in shim (tfhe-gpu_amd/shim/bootstrapping_hip.cpp -> the seven boundary
                symbols): end-to-end bootstraps/s of the unchanged caller, the shim's own time per
                call, and its outputs checked against the benchmarked device-resident outputs.
  cpu_baseline  the REFERENCE's own OpenFHE CPU path (oracle/_ref/ref_kat: the unchanged vector
                API with the reference's CPU accumulator and key switch behind the GPU symbols,
                OpenMP over ciphertexts) on a bounded sample of the same workload with the same
                context and keys on this host's cores (rank 0, N = 1 only), which also checks the
                benchmarked GPU outputs bit for bit; the C restatement (oracle/) only when ref_kat
                is absent (then kind "port" and "fallback" says why).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))

MIB = 1 << 20
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md chip table (spec)
VALU_CYCLES = 4                    # cycles per wave64 VALU instruction (mul/mad class; profiles/r01_valu_rates.txt)
CLOCK_HZ = 2.4e9                   # MI355X peak engine clock
SIGN_MOD = 1 << 23                 # C5: Encrypt(sk, m, FRESH, p, Qin = 2^23)

# SURVEY.md 8(d).  ctx: ("set", name) or ("logq", name, arbFunc, logQ, N, baseG, throw) as
# GenerateBinFHEContext; ref: the same context for oracle/_ref/ref_kat; per_unit_s: one unit (gate,
# EvalFunc or EvalSign) of the reference's CPU path on one GPU-box core (sizes the CPU sample only).
CONFIGS = {
    "C2": {"ctx": ("set", "STD128"), "op": "gate", "batch": 8192, "scaling": "weak", "ref": "set:STD128",
           "per_unit_s": 0.12, "what": "STD128 GINX EvalBinGate(NAND)"},
    "C3": {"ctx": ("logq", "STD128", True, 12, 0, 0, 1), "op": "func", "batch": 4096, "scaling": "weak",
           "ref": "logq:STD128,1,12,0,0,1", "per_unit_s": 1.6,
           "what": "STD128 arbFunc logQ=12 throw=1 EvalFunc(x^3 mod 8), arbitrary LUT"},
    "C4": {"ctx": ("set", "STD192"), "op": "gate", "batch": 8192, "scaling": "weak", "ref": "set:STD192",
           "per_unit_s": 0.5, "what": "STD192 GINX EvalBinGate(NAND)"},
    "C5a": {"ctx": ("set", "STD128Q"), "op": "sign", "batch": 1024, "scaling": "strong", "ref": "set:STD128Q",
            "per_unit_s": 6.5, "what": "STD128Q EvalSign, ciphertext modulus 2^23"},
    "C5b": {"ctx": ("logq", "STD128", False, 23, 0, 0, 1), "op": "sign", "batch": 1024, "scaling": "strong",
            "ref": "logq:STD128,0,23,0,0,1", "per_unit_s": 4.0,
            "what": "STD128 logQ=23 throw=1 EvalSign, ciphertext modulus 2^23"},
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS), help="SURVEY.md 8(d) configuration")
    ap.add_argument("--batch", type=int, default=0,
                    help="ciphertexts per GPU (weak scaling) or in all (strong scaling); 0 = the config's")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="weak: --batch per GPU (C2-C4's default: BASELINE's 'batch=8192 at 1/2/4/8 GPUs' read as "
                         "8192 per GPU); strong: --batch in all, sharded over the GPUs (C5's default; C2 strong = "
                         "8192 in all, 8192/N per GPU)")
    ap.add_argument("--params", default=None,
                    help="EvalBinGate(NAND) on another parameter set (e.g. STD192, STD128Q): device-resident, "
                         "no cpu_baseline (overrides --config's context)")
    ap.add_argument("--kernel-reps", type=int, default=2, help="blind-rotation launches timed for the roofline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--generic", action="store_true", help="force the generic LDS blind-rotation kernel")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend ('nccl' = RCCL; 'gloo' only to rehearse N ranks on fewer GPUs)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline sample length")
    ap.add_argument("--pmc-json", default=None, help="PMC record of the blind rotation (default: per config)")
    ap.add_argument("--valu-peak-json", default=None, help="VALU peak record (default: the newest)")
    ap.add_argument("--no-host-array", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the reference-through-the-shim leg")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="launch knob (tfhe_knobs) for A/B runs; repeatable")
    ap.add_argument("--test-lib", action="store_true",
                    help="run on lib/libtfhe_hip_test.so (fault-probe / timing builds; A/B runs only)")
    return ap.parse_args()


def newest(*paths):
    for p in paths:
        if os.path.exists(p):
            return p
    return paths[0]


GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix_stream(seed, start, count, mod, out):
    """out[k] = splitmix64 value number start+k+1 of seed, mod `mod` (SURVEY.md Appendix B
    generator; the stream or_kat_keys and the reference driver draw from), vectorised."""
    M1, M2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)
    step = 1 << 24
    with np.errstate(over="ignore"):
        for o in range(0, count, step):
            k = np.arange(start + o + 1, start + min(count, o + step) + 1, dtype=np.uint64)
            z = np.uint64(seed) + k * GAMMA
            z = (z ^ (z >> np.uint64(30))) * M1
            z = (z ^ (z >> np.uint64(27))) * M2
            z ^= z >> np.uint64(31)
            out[o:o + len(k)] = z % np.uint64(mod)
    return out


def synthetic_keys(p, seed=1):
    """The Appendix B synthetic keys ("synth:<seed>": BSK coefficients then KSK words from one
    splitmix64 stream), so the reference CPU run (cpu_baseline) uses exactly the same keys;
    throughput does not depend on key validity."""
    nb, nk = p.bsk_words(), p.ksk_words()
    bsk = splitmix_stream(seed, 0, nb, p.Q, np.empty(nb, dtype=np.uint64))
    ksk = splitmix_stream(seed, nb, nk, p.qKS, np.empty(nk, dtype=np.uint64))
    return bsk, ksk


def modmuls_per_bootstrap(p):
    """n[(dG2+2)(N/2)log2N + 4 dG2 N + 4N]."""
    logN = p.N.bit_length() - 1
    return p.n * ((p.dG2 + 2) * (p.N // 2) * logN + 4 * p.dG2 * p.N + 4 * p.N)


def b_alg_per_bootstrap(p):
    """BSK packed (u32 if Q < 2^32) + KS gather (packed) + LWE I/O."""
    wb = 4 if p.Q < (1 << 32) else 8
    kb = 2 if p.qKS <= (1 << 16) else (4 if p.qKS <= (1 << 32) else 8)
    bsk = p.n * 2 * p.dG2 * 2 * p.N * wb
    ks = p.N * p.dKS * (p.n + 1) * kb
    io = 3 * (p.n + 1) * 8
    return bsk + ks + io, bsk


def peak_family(br_kernel, p):
    """The product the context's blind rotation issues (tfhe_info.br_kernel) -> valu_peak.json family."""
    if br_kernel == 1:
        return "smont_i32"                                 # blind_rotate_fast4.hip
    if br_kernel in (2, 3):
        return "fmod_q37" if p.Q < (1 << 40) else "fmod_q50"  # blind_rotate_f64.hip
    if br_kernel == 5:
        return "sf_q54"                                    # sf2 / gen3sf, blind_rotate_generic.hip
    return None


def host_threads():
    """Threads for the CPU baseline: every core this process may run on, unless the pool caps
    OpenMP (OMP_NUM_THREADS is set to the box's CPU share on the GPU pool)."""
    visible = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(visible, cap) if cap else visible), visible


REF_KAT = os.path.join(ROOT, "oracle", "_ref", "ref_kat")
REF_DROPIN = os.path.join(ROOT, "oracle", "_ref", "ref_dropin")


def cube_lut(q, P=8):
    """GenerateLUTviaFunction(m^3 mod p, p) (binfhecontext.cpp:280-301; time-estimate.cpp:70-75), the
    C3 LUT (tests/test_oracle_ref_vectors.py pins it to the reference's own)."""
    interval = q // P

    def f(m, p1):
        return (m * m * m) % p1 if m < p1 else ((m - p1 // 2) ** 3) % p1

    return np.array([f(i // interval, P) * interval for i in range(q)], dtype=np.uint64)


def dropin_leg(h1, h2, want, host_array_ms, reps=3):
    """The reference's unchanged vector EvalBinGate(NAND) on this GPU through the shim,
    on the benchmarked inputs with the same synthetic keys ("synth:1" = synthetic_keys)."""
    import re
    import subprocess
    import tempfile

    if not os.path.exists(REF_DROPIN):
        return None
    B = len(h1)
    with tempfile.TemporaryDirectory() as tmp:
        f1, f2, fo = (os.path.join(tmp, x) for x in ("c1", "c2", "out"))
        h1.tofile(f1)
        h2.tofile(f2)
        env = dict(os.environ, TFHE_SHIM_TIMING="1")
        r = subprocess.run([REF_DROPIN, "ctx=set:STD128", "keys=synth:1", "op=NAND", "api=vector", "gpus=1",
                            f"in={f1}", f"in2={f2}", f"out={fo}", f"reps={reps}"],
                           capture_output=True, text=True, env=env, timeout=600)
        if r.returncode:
            raise RuntimeError(r.stderr[-2000:])
        js = json.loads(r.stdout.strip().splitlines()[-1])
        out = np.fromfile(fo, dtype=np.uint64).reshape(B, -1)
    phases = {}
    for m in re.finditer(r"\[shim\] (\w+) (.+?) B=(\d+) ([\d.]+) ms", r.stderr):
        if int(m.group(3)) == B:
            phases.setdefault(f"{m.group(1)} {m.group(2)}", []).append(float(m.group(4)))
    # per call: the fastest rep of each phase (the first rep carries first-touch costs)
    shim_ms = sum(min(v) for k, v in phases.items() if not k.startswith("GPUSetup"))
    return {"value": round(B / js["best_s"], 1), "unit": "bootstraps/s", "best_ms": round(js["best_s"] * 1e3, 3),
            "shim_ms": round(shim_ms, 3), "shim_vs_host_array": round(shim_ms / host_array_ms, 3),
            "reference_glue_ms": round(js["best_s"] * 1e3 - shim_ms, 3),
            "equal_to_device_resident": bool(np.array_equal(out, want)),
            "note": "oracle/_ref/ref_dropin: the reference's BinFHEContext::EvalBinGate(vector) unchanged, its "
                    "seven GPU symbols served by the shim over libtfhe_hip.so, same keys and inputs; value = "
                    "end to end incl. the reference's own single-threaded host glue (reference_glue_ms); "
                    "shim_ms = the shim's marshalling + device time per call (fastest of the reps per phase)"}


def ref_call_args(cfg, p, files):
    """ref_kat arguments for the config's op on the input files (in, in2, lut)."""
    if cfg["op"] == "gate":
        return ["op=NAND", f"in={files['in']}", f"in2={files['in2']}"]
    if cfg["op"] == "func":
        return ["op=func", f"in={files['in']}", f"lut={files['lut']}", f"mod={p.q}"]
    return ["op=sign", f"in={files['in']}", f"mod={SIGN_MOD}"]


def cpu_baseline_reference(name, cfg, p, seconds, gpu_sample, bs_per_unit):
    """The reference's own OpenFHE code (oracle/_ref/ref_kat: the vector API, CPU functions behind the
    seven GPU symbols, OpenMP over ciphertexts) on K units of the same context with the same keys; the
    first ones are the GPU's benchmarked inputs, whose outputs are compared bit for bit."""
    import subprocess
    import tempfile

    threads, visible = host_threads()
    ins, gout = gpu_sample["in"], gpu_sample["out"]
    per = cfg["per_unit_s"]
    K = max(len(gout), threads * max(1, int(seconds / per)))
    rs = np.random.default_rng(5)
    width = p.n + 1
    mod = SIGN_MOD if cfg["op"] == "sign" else p.q
    arrs = {k: np.concatenate([v, rs.integers(0, mod, (K - len(v), width), dtype=np.uint64)]) for k, v in ins.items()}

    # one process, one key load: first a 1-thread sample of B1 units (the single-thread figure SURVEY 8(d)
    # asks for), then all K units on `threads` threads (ref_kat sizes= / threads=); the output is the last run's
    B1 = min(K, max(2, int(seconds / 4 / per)))
    with tempfile.TemporaryDirectory() as tmp:
        files = {}
        for k, v in arrs.items():
            files[k] = os.path.join(tmp, k)
            v[:K].tofile(files[k])
        if cfg["op"] == "func":
            files["lut"] = os.path.join(tmp, "lut")
            cube_lut(p.q).tofile(files["lut"])
        fo = os.path.join(tmp, "out")
        env = dict(os.environ, OMP_NUM_THREADS=str(threads))
        r = subprocess.run([REF_KAT, f"ctx={cfg['ref']}", "keys=synth:1", "api=vector", f"out={fo}",
                            f"sizes={B1},{K}", f"threads=1,{threads}"]
                           + ref_call_args(cfg, p, files), capture_output=True, text=True, env=env, timeout=1800)
        if r.returncode:
            raise RuntimeError(r.stderr[-2000:])
        js = json.loads(r.stdout.strip().splitlines()[-1])
        out = np.fromfile(fo, dtype=np.uint64).reshape(K, width)
    sw1, swK = js["sweep"]
    assert (sw1["B"], sw1["threads"], swK["B"], swK["threads"]) == (B1, 1, K, threads), js["sweep"]
    js["best_s"] = swK["best_s"]
    single = round(B1 * bs_per_unit / sw1["best_s"], 3)
    parity = {"ciphertexts": int(len(gout)), "bit_exact": bool(np.array_equal(out[:len(gout)], gout)),
              "vs": "the reference's OpenFHE CPU path (oracle/_ref/ref_kat), same context, keys and inputs"}
    unit = {"gate": "EvalBinGate(NAND)", "func": "EvalFunc", "sign": "EvalSign"}[cfg["op"]]
    return {"value": round(K * bs_per_unit / js["best_s"], 3), "unit": "bootstraps/s", "cores": threads,
            "kind": "reference", "host_cores_visible": visible, "single_thread_value": single,
            "sample": f"{cfg['what']}: the vector API of the reference's OpenFHE (compiled from its sources, "
                      f"oracle/Makefile.ref) with its CPU accumulator / key switch behind the GPU symbols, OpenMP "
                      f"over ciphertexts, {threads} threads: {K} x {unit} ({bs_per_unit} bootstraps each) in "
                      f"{js['best_s']:.1f} s (key load {js['key_load_s']:.1f} s not counted); single thread: "
                      f"{B1} units in {sw1['best_s']:.1f} s",
            "gpu_parity": parity}


SAMPLE_PER_RANK = {"gate": 8, "func": 2, "sign": 1}   # ciphertexts of every rank's shard checked by the oracle


def oracle_params(cfg):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    spec = cfg["ctx"]
    return pyoracle.params_from_set(spec[1]) if spec[0] == "set" else pyoracle.params_from_logq(spec[1], *spec[2:])


def gather_rank_samples(arrs, world, dev):
    """Every rank's sample arrays (same shape on every rank) in rank order, on every rank."""
    if world == 1:
        return [arrs]
    import torch
    import torch.distributed as dist

    flat = np.concatenate([a.reshape(-1) for a in arrs]).astype(np.int64)
    t = torch.from_numpy(flat).to(dev)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    res = []
    for o in outs:
        v = o.cpu().numpy().astype(np.uint64)
        parts, off = [], 0
        for a in arrs:
            parts.append(v[off:off + a.size].reshape(a.shape))
            off += a.size
        res.append(parts)
    return res


def oracle_sample_check(cfg, bsk, ksk, per_rank, lut=None, threads=0):
    """The C restatement (oracle/tfhe_oracle.c, the allowed checker) on every rank's sample:
    per_rank = [[in1, (in2,) out] per rank].  Returns the record the bench line carries."""
    t0 = time.perf_counter()
    op = oracle_params(cfg)
    import pyoracle

    orc = pyoracle.Oracle(op, bsk, ksk, threads=threads)
    passed = []
    try:
        for arrs in per_rank:
            if cfg["op"] == "gate":
                ref = orc.eval_bin_gate("NAND", arrs[0], arrs[1])
            elif cfg["op"] == "func":
                ref = orc.eval_func(arrs[0], lut)
            else:
                ref = orc.eval_sign(arrs[0], SIGN_MOD)
            passed.append(bool(np.array_equal(ref, arrs[-1])))
    finally:
        orc.close()
    return {"ranks_checked": len(per_rank), "ranks_passed": int(sum(passed)), "per_rank": passed,
            "ciphertexts_per_rank": int(len(per_rank[0][-1])), "seconds": round(time.perf_counter() - t0, 2),
            "vs": "oracle/tfhe_oracle.c (C restatement of the reference's CPU path) on the first ciphertexts "
                  "of every rank's benchmarked shard, same synthetic keys, outside the timed region"}


def parity_verdict(cpu, host_array, dropin, oracle):
    """(ok, failed checks) over every output check the line carries; a check that did not run is not
    a failure, one that ran and disagreed is."""
    failed = []
    if cpu and cpu.get("gpu_parity") and not cpu["gpu_parity"]["bit_exact"]:
        failed.append("cpu_baseline.gpu_parity")
    if host_array and not host_array.get("equal_to_device_resident", True):
        failed.append("host_array.equal_to_device_resident")
    if dropin and not dropin.get("equal_to_device_resident", True):
        failed.append("dropin.equal_to_device_resident")
    if oracle is None:
        failed.append("oracle_sample (did not run)")
    elif oracle.get("ranks_passed") != oracle.get("ranks_checked"):
        failed.append("oracle_sample")
    return not failed, failed


def cpu_baseline_port(p, bsk, ksk, seconds, gpu_sample, reason):
    """Fallback when oracle/_ref/ref_kat is absent: the C restatement (oracle/tfhe_oracle.c), STD128 NAND."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    pyoracle.build()
    threads, visible = host_threads()
    orc = pyoracle.Oracle(pyoracle.params_from_set("STD128"), bsk, ksk, threads=threads)
    rs = np.random.default_rng(5)
    B0 = threads
    c1 = rs.integers(0, p.q, (B0, p.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, p.q, (B0, p.n + 1), dtype=np.uint64)
    t0 = time.perf_counter()
    orc.eval_bin_gate("NAND", c1, c2)
    t_cal = time.perf_counter() - t0
    B = B0 * max(1, int(seconds / max(t_cal, 1e-3)))
    c1 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    t0 = time.perf_counter()
    orc.eval_bin_gate("NAND", c1, c2)
    dt = time.perf_counter() - t0
    orc.L.or_set_threads(1)
    B1 = max(1, int(seconds / 4 / max(t_cal, 1e-3)))
    t0 = time.perf_counter()
    orc.eval_bin_gate("NAND", c1[:B1], c2[:B1])
    dt1 = time.perf_counter() - t0
    orc.L.or_set_threads(threads)
    g1, g2 = gpu_sample["in"]["in"], gpu_sample["in"]["in2"]
    ref = orc.eval_bin_gate("NAND", g1, g2)
    parity = {"ciphertexts": int(len(g1)), "bit_exact": bool(np.array_equal(ref, gpu_sample["out"])),
              "vs": "oracle/tfhe_oracle.c on the same synthetic keys and inputs"}
    orc.close()
    return {"value": round(B / dt, 3), "unit": "bootstraps/s", "cores": threads, "kind": "port",
            "host_cores_visible": visible, "single_thread_value": round(B1 / dt1, 3), "fallback": reason,
            "sample": f"STD128 EvalBinGate(NAND) on {B} random ciphertext pairs, same synthetic keys; "
                      f"oracle/tfhe_oracle.c (exact u128 CPU restatement, OpenMP one ciphertext per thread); "
                      f"{dt:.1f} s; single thread: {B1} pairs in {dt1:.1f} s",
            "gpu_parity": parity}


def batch_split(cfg, batch, world, rank):
    """(this rank's batch, the whole job's): weak scaling = `batch` per GPU, strong = `batch` in all, cut into
    contiguous shards (tfhe_shard_range)."""
    from tfhe_amd import dist as tdist

    if cfg["scaling"] == "strong":
        lo, hi = tdist.shard_range(batch, world, rank)
        return hi - lo, batch
    return batch, batch * world


def metric_name(name, cfg, total, B, world, params=False):
    """BASELINE.json's metric with the reading stated: the global batch, and per-GPU batch (weak) or the
    shard count (strong)."""
    what = f"{cfg['ctx'][1]} GINX" if name == "C2" or params else f"{name}: {cfg['what']},"
    how = (f"{B} per GPU, weak scaling" if cfg["scaling"] == "weak"
           else f"sharded over {world} GPU{'s' if world > 1 else ''}, strong scaling")
    return f"bootstraps/sec (whole node), {what} global batch={total} ({how})"


def main():
    args = parse()
    name = args.config
    cfg = dict(CONFIGS[name])
    if args.params:
        cfg.update(ctx=("set", args.params), op="gate", what=f"{args.params} GINX EvalBinGate(NAND)", ref=None,
                   scaling="weak")
        name = args.params
        args.no_cpu_baseline = True
    if args.generic:
        os.environ["TFHE_FORCE_GENERIC"] = "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU "
              f"(torch.distributed.run --nproc-per-node {args.gpus})", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist
    import tfhe_amd
    from tfhe_amd import dist as tdist

    local_dev = local % max(1, torch.cuda.device_count())  # == local on a full node
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    ctxspec = cfg["ctx"]
    p = (tfhe_amd.params_from_set(ctxspec[1]) if ctxspec[0] == "set"
         else tfhe_amd.params_from_logq(ctxspec[1], *ctxspec[2:]))
    if args.scaling:
        cfg["scaling"] = args.scaling
    B, total = batch_split(cfg, args.batch or cfg["batch"], world, rank)
    # a dedicated (non-null) stream: the engine's kernels, torch's tensors and the
    # HIP events below are all ordered on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    # ---- GPUSetup: rank 0 converts the keys, the image is broadcast over RCCL ----
    t_setup = time.perf_counter()
    bcast_ms = None
    libpath = tfhe_amd.capi.TEST_LIB if args.test_lib else None
    knobs = {k: int(v) for k, v in (x.split("=", 1) for x in args.knob)}
    if rank == 0:
        bsk, ksk = synthetic_keys(p)
        ctx = tfhe_amd.BinFHEContextHIP(p, library=libpath).GPUSetup(bsk, ksk)
        # large host keys are not held through the timed run (C3 / C5b: a 4.8 GB KSK); the oracle check and the
        # port fallback regenerate them deterministically (synthetic_keys) after it
        if bsk.nbytes + ksk.nbytes > (3 << 30):
            bsk = ksk = None
    else:
        bsk = ksk = None
    if world > 1:
        # one RCCL broadcast of the packed device key image over xGMI (tfhe_amd/dist.py)
        img = None
        nbytes = ctx.info().key_image_bytes if rank == 0 else None
        if rank == 0:
            img = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            ctx.export_key_image(img.data_ptr(), nbytes, sptr)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        img = tdist.broadcast_key_image(img, nbytes, dev)
        torch.cuda.synchronize(dev)
        bcast_ms = (time.perf_counter() - t0) * 1e3
        if rank != 0:
            ctx = tfhe_amd.BinFHEContextHIP.from_key_image(p, img.data_ptr(), img.numel(), local_dev, libpath)
        del img
        bcast_ms = tdist.max_over_ranks(bcast_ms, dev)
    setup_s = time.perf_counter() - t_setup
    if knobs:
        ctx.set_knobs(**knobs)

    # ---- inputs resident in HBM ----
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    in_mod = SIGN_MOD if cfg["op"] == "sign" else int(p.q)
    ct1 = torch.randint(0, in_mod, (B, p.n + 1), dtype=torch.int64, device=dev, generator=g)
    ct2 = torch.randint(0, in_mod, (B, p.n + 1), dtype=torch.int64, device=dev, generator=g)
    out = torch.empty((B, p.n + 1), dtype=torch.int64, device=dev)
    lut = torch.from_numpy(cube_lut(int(p.q)).astype(np.int64)).to(dev) if cfg["op"] == "func" else None

    def step():
        if cfg["op"] == "gate":
            ctx.EvalBinGateDevice("NAND", B, ct1.data_ptr(), ct2.data_ptr(), out.data_ptr(), stream=sptr)
        elif cfg["op"] == "func":
            ctx.EvalFuncDevice(B, ct1.data_ptr(), lut.data_ptr(), out.data_ptr(), stream=sptr)
        else:
            ctx.EvalSignDevice(B, ct1.data_ptr(), SIGN_MOD, out.data_ptr(), stream=sptr)

    b0 = ctx.info().bootstraps
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    bs_per_unit = (ctx.info().bootstraps - b0) // (max(1, args.warmup) * B)  # the engine's own count
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = tdist.max_over_ranks(elapsed, dev)
    total_bs = total * bs_per_unit * args.steps
    value = total_bs / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- dominant kernel (blind rotation) timed alone with HIP events on its stream ----
    a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
    acc = torch.zeros((B, 2, p.N), dtype=torch.int64, device=dev)
    acc[:, 1, ::2] = int(p.Q // 8 + 1)
    lib = tfhe_amd.lib()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    tfhe_amd.capi.check(lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sptr),
                        "tfhe_eval_acc_device")
    e0.record(stream)
    for _ in range(args.kernel_reps):
        tfhe_amd.capi.check(lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sptr),
                            "tfhe_eval_acc_device")
    e1.record(stream)
    torch.cuda.synchronize(dev)
    br_ms = e0.elapsed_time(e1) / args.kernel_reps
    rank_ms = tdist.gather_over_ranks(br_ms, dev) if world > 1 else [br_ms]
    info = ctx.info()
    balg, bsk_bytes = b_alg_per_bootstrap(p)
    pmc_json = args.pmc_json or newest(os.path.join(ROOT, "profiles", f"r06_pmc_{name}.json"),
                                       os.path.join(ROOT, "profiles", f"r05_pmc_{name}.json"),
                                       os.path.join(ROOT, "profiles", f"r04_pmc_{name}.json"),
                                       *([os.path.join(ROOT, "profiles", "r03_pmc_blind_rotate.json")]
                                         if name == "C2" else []))
    traffic, valu_insts, pmc = None, None, {}
    if os.path.exists(pmc_json):
        try:
            pmc = json.load(open(pmc_json))
            if pmc.get("units_per_launch") == B:
                traffic = pmc.get("hbm_bytes_per_launch")
                valu_insts = pmc.get("sq_insts_valu_per_launch")
            else:
                pmc = {}
        except Exception:
            traffic, valu_insts, pmc = None, None, {}
    mm = modmuls_per_bootstrap(p)
    achieved_mm = mm * B / (br_ms * 1e-3)
    fam = peak_family(int(info.br_kernel), p)
    vp_json = args.valu_peak_json or newest(os.path.join(ROOT, "profiles", "r04_valu_peak.json"),
                                            os.path.join(ROOT, "profiles", "r03_valu_peak.json"))
    peak_mm, peak_clock, peak_label = None, None, None
    if os.path.exists(vp_json) and fam:
        vp = json.load(open(vp_json))
        pk = vp.get("peaks", {}).get(fam)
        if pk is None and fam == "smont_i32":  # a round-3 record (smont only)
            pk = {"modmul_per_s": vp["modmul_per_s"], "held_clock_ghz": vp.get("held_clock_ghz"),
                  "kernel": vp.get("kernel")}
        if pk:
            peak_mm, peak_clock, peak_label = pk["modmul_per_s"], pk.get("held_clock_ghz"), pk.get("kernel")
    roofline = {"bound": "valu-int", "achieved": round(achieved_mm / 1e12, 3),
                "peak": None if peak_mm is None else round(peak_mm / 1e12, 3), "unit": "Tmodmul/s",
                "frac": None if peak_mm is None else round(achieved_mm / peak_mm, 3), "traffic": traffic,
                "kernel": "blind_rotate (tfhe_eval_acc_device)", "kernel_ms": round(br_ms, 3),
                "units_per_launch": B, "alg_modmul_per_unit": mm, "peak_family": fam,
                "hbm_frac": None if traffic is None else round(traffic / (br_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4),
                "effective_keystream_tbs": round(balg * B / (br_ms * 1e-3) / 1e12, 2), "alg_bytes_per_unit": balg,
                "note": "achieved = SURVEY 8(d) algorithmic modmuls per bootstrap x batch / event-timed kernel; peak = "
                        f"the microbenchmarked rate of the product this kernel issues ({peak_label}, "
                        + os.path.relpath(vp_json, ROOT) + (f", held {peak_clock} GHz" if peak_clock else "")
                        + "); hbm_frac = PMC HBM bytes / kernel time / 8 TB/s; effective_keystream_tbs = B_alg "
                          "(no cross-ciphertext reuse) x batch / kernel time, served from L2/MALL"}
    simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
    valu = {"bound": "valu-int", "modmul_per_bootstrap": mm,
            "achieved_modmul_per_s": round(mm * B / (br_ms * 1e-3), 1),
            "valu_instr_per_launch": valu_insts,
            "issue_frac": None if valu_insts is None else
            round(valu_insts * VALU_CYCLES / (simds * CLOCK_HZ * br_ms * 1e-3), 3),
            "note": "issue_frac (mixed-unit: 4 cycles per VALU instruction at 2.4 GHz; quote busy_frac) from "
                    + os.path.relpath(pmc_json, ROOT)}
    act, gui = pmc.get("sq_active_inst_valu_per_launch"), pmc.get("grbm_gui_active_per_launch")
    if act and gui:
        # measured in one PMC pass, clock-independent: VALU-executing cycles per SIMD over the
        # launch's cycles (GRBM_GUI_ACTIVE sums the 8 XCDs; SQ_ACTIVE_INST_VALU is quad-cycles)
        valu["busy_frac"] = round(act * 4 / simds / (gui / 8), 3)
        pass_ns = pmc.get("gui_pass_kernel_ns_per_launch")  # the GUI pass's own dispatch time
        valu["held_clock_ghz"] = round(gui / 8 / (pass_ns * 1e-9 if pass_ns else br_ms * 1e-3) / 1e9, 2)
        valu["note"] += ("; busy_frac = SQ_ACTIVE_INST_VALU x 4 / SIMDs / (GRBM_GUI_ACTIVE / 8); held_clock_ghz = "
                         "GRBM_GUI_ACTIVE / 8 / kernel time (profiled pass, MI355X_MICROARCH.md 'DVFS give-back')")
        if peak_mm and peak_clock:
            # the same peak scaled to the clock the part holds under this kernel (power-limited): how much
            # of the gap is issue efficiency and how much is clock
            peak_k = peak_mm * valu["held_clock_ghz"] / peak_clock
            roofline["frac_at_kernel_clock"] = round(achieved_mm / peak_k, 3)
            roofline["note"] += (f"; frac_at_kernel_clock = achieved / (peak x {valu['held_clock_ghz']} GHz held under "
                                 f"the kernel / {peak_clock} GHz held under the microbenchmark)")

    # ---- the same op through the host-array entry point (PCIe + host staging included), every rank ----
    host_array = None
    out_h = out.cpu().numpy().astype(np.uint64)
    h1 = ct1.cpu().numpy().astype(np.uint64)
    h2 = ct2.cpu().numpy().astype(np.uint64)
    if not args.no_host_array:
        lut_h = cube_lut(int(p.q)) if cfg["op"] == "func" else None

        def host_call():
            if cfg["op"] == "gate":
                return ctx.EvalBinGate("NAND", h1, h2)
            if cfg["op"] == "func":
                return ctx.EvalFunc(h1, lut_h)
            return ctx.EvalSign(h1, SIGN_MOD)

        best = None
        for _ in range(2):
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            hout = host_call()
            dt = time.perf_counter() - t0
            if world > 1:
                dt = tdist.max_over_ranks(dt, dev)
            best = dt if best is None else min(best, dt)
        host_array = {"value": round(total * bs_per_unit / best, 1), "unit": "bootstraps/s", "ms": round(best * 1e3, 3),
                      "equal_to_device_resident": bool(np.array_equal(hout, out_h)),
                      "note": "host arrays in and out (tfhe_eval_bin_gate / _func / _sign): H2D + kernels + D2H "
                              "through pinned staging, best of 2, slowest rank"}
        if world > 1:
            host_array["equal_to_device_resident"] = bool(tdist.sum_over_ranks(
                int(not host_array["equal_to_device_resident"]), dev) == 0)

    dropin = None
    if rank == 0 and world == 1 and name == "C2" and not args.no_dropin and host_array is not None:
        try:
            dropin = dropin_leg(h1, h2, out_h, host_array["ms"])
        except Exception as e:  # reported, never fatal: the headline does not depend on it
            print(f"[bench] drop-in leg failed: {e}", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        K = min(B, 64 if cfg["op"] == "gate" else 16)
        sample = {"in": {"in": h1[:K]} if cfg["op"] != "gate" else {"in": h1[:K], "in2": h2[:K]}, "out": out_h[:K]}
        reason = None
        if os.path.exists(REF_KAT):
            try:
                cpu = cpu_baseline_reference(name, cfg, p, args.cpu_seconds, sample, bs_per_unit)
            except Exception as e:
                reason = f"oracle/_ref/ref_kat failed: {e}"
        else:
            reason = ("oracle/_ref/ref_kat absent (built only where /root/reference exists: oracle/Makefile.ref; "
                      "git-ignored, it reaches the GPU box with the working tree)")
        if cpu is None:
            print(f"[bench] reference CPU baseline unavailable ({reason}); using the C restatement", file=sys.stderr)
            if name == "C2":
                if bsk is None:
                    bsk, ksk = synthetic_keys(p)
                cpu = cpu_baseline_port(p, bsk, ksk, args.cpu_seconds, sample, reason)

    # ---- every rank's shard: its first ciphertexts against the C restatement (rank 0 checks all) ----
    ks = min(B, SAMPLE_PER_RANK[cfg["op"]])
    mine = [h1[:ks]] + ([h2[:ks]] if cfg["op"] == "gate" else []) + [out_h[:ks]]
    per_rank = gather_rank_samples(mine, world, dev)
    oracle = None
    if rank == 0 and not args.params:
        try:
            if bsk is None:
                bsk, ksk = synthetic_keys(p)
            oracle = oracle_sample_check(cfg, bsk, ksk, per_rank,
                                         lut=cube_lut(int(p.q)) if cfg["op"] == "func" else None,
                                         threads=host_threads()[0])
        except Exception as e:
            print(f"[bench] oracle sample check failed to run: {e}", file=sys.stderr)
    elif rank == 0:
        oracle = {"skipped": "--params: no oracle context for an ad-hoc parameter run", "ranks_checked": 0,
                  "ranks_passed": 0}
    parity_ok, failed = parity_verdict(cpu, host_array, dropin, oracle) if rank == 0 else (True, [])
    if world > 1:  # rank 0's verdict is every rank's exit status
        parity_ok = tdist.max_over_ranks(0.0 if parity_ok else 1.0, dev) == 0.0
    if rank == 0 and not parity_ok:
        print(f"[bench] ERROR: output checks failed: {', '.join(failed)}", file=sys.stderr)

    if rank == 0:
        line = {
            "metric": metric_name(name, cfg, total, B, world, bool(args.params)),
            "value": round(value, 2), "unit": "bootstraps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": cfg["scaling"], "vs_baseline": None, "data": "synthetic",
            "dtype": {0: "u32" if int(info.word_bits) == 32 else "u64", 1: "u32", 2: "f64",
                      3: "f64", 4: "i32", 5: "u64"}[int(info.br_kernel)],
            "config": {"workload": f"{name}: {cfg['what']}, inputs resident in HBM", "config": name,
                       "global_batch": total, "batch_per_gpu": B, "bootstraps_per_unit": bs_per_unit,
                       "n": p.n, "N": p.N, "Q": p.Q, "dG2": p.dG2, "parallelism": f"shard{world}"},
            "value_end_to_end": None if host_array is None else host_array["value"],
            "dist": {"backend": dist.get_backend() if world > 1 else None,
                     "world_size": dist.get_world_size() if world > 1 else 1,
                     "kernel_ms_max": round(max(rank_ms), 3), "kernel_ms_min": round(min(rank_ms), 3),
                     "key_broadcast_ms": None if bcast_ms is None else round(bcast_ms, 2)},
            "parity_ok": parity_ok, "parity_failed": failed, "oracle_sample": oracle,
            "roofline": roofline, "valu": valu, "host_array": host_array, "dropin": dropin, "cpu_baseline": cpu,
            "setup_s": round(setup_s, 2), "key_broadcast_ms": None if bcast_ms is None else round(bcast_ms, 2),
            "key_image_bytes": int(info.key_image_bytes),
        }
        if knobs or args.test_lib:
            line["knobs"] = dict(knobs, test_lib=args.test_lib)
        print(json.dumps(line), flush=True)
    ctx.GPUClean()
    if world > 1:
        dist.destroy_process_group()
    return 0 if parity_ok else 1


if __name__ == "__main__":
    sys.exit(main())
