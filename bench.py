#!/usr/bin/env python3
"""bench.py -- bootstraps/sec of the batched STD128 GINX bootstrap on MI355X.

Workload (BASELINE.json configs[1]): STD128 (n=512, N=1024, Q=2^27-2^11+1,
baseG=2^7) EvalBinGate(NAND), batch 8192 per GPU.  One step = one vector
EvalBinGate call over the batch with both input vectors already resident in HBM:
test vector -> blind rotation (n external products) -> extraction -> MKM, all on
device (the fused tfhe_eval_bin_gate_device entry point).  One bootstrap per gate.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU; the key image is built once on rank 0 and broadcast over
RCCL/xGMI (torch.distributed, backend "nccl" = RCCL), then every rank bootstraps
its own 8192-ciphertext shard with no data-path collective (weak scaling).

Extra JSON fields:
  roofline      the blind-rotation kernel (the dominant one), timed alone with HIP
                events on its stream.  Its bound is integer VALU issue:
                bound "valu-int", achieved = the algorithmic modular multiplies of
                SURVEY 8(d) (n[(dG2+2)(N/2)log2 N + 4 dG2 N + 4N] per bootstrap) per
                second, peak = the microbenchmarked signed-Montgomery modmul rate of
                gfx950 (tools/microbench/valu_rates.hip, --valu-peak-json), frac = their
                ratio.  traffic = PMC HBM bytes per launch (rocprofv3 FETCH_SIZE x2 +
                WRITE_SIZE, MI355X_MICROARCH.md corrections; --pmc-json), hbm_frac =
                traffic / kernel time / 8 TB/s, effective_keystream_tbs = SURVEY B_alg
                (BSK + KS gather + LWE I/O per bootstrap, no cross-ciphertext reuse) x
                batch / kernel time.
  valu          PMC view of the same kernel: VALU instructions, issue and busy
                fractions, the clock the part held under it.
  host_array    the same gates through the host-array entry point (tfhe_eval_bin_gate:
                PCIe copies, pinned staging and the host thread included), same inputs.
  dropin        the reference's own, unchanged vector EvalBinGate (OpenFHE BinFHE code compiled from
                its sources, oracle/_ref/ref_dropin) running on this GPU through the drop-in shim
                (tfhe-gpu_amd/shim/bootstrapping_hip.cpp -> the seven boundary symbols): end-to-end
                bootstraps/s of the unchanged caller, the shim's own time per call (marshalling +
                device, TFHE_SHIM_TIMING) against the host-array API, and its outputs checked
                against the benchmarked device-resident outputs (same keys, same inputs).
  cpu_baseline  the REFERENCE's own OpenFHE CPU path (oracle/_ref/ref_kat: the
                unchanged vector EvalBinGate with the reference's CPU accumulator and
                key switch behind the GPU symbols, OpenMP over ciphertexts) on a bounded
                sample of the same workload with the same keys on this host's cores
                (rank 0, N = 1 only), which also checks the benchmarked GPU outputs bit
                for bit; the C restatement (oracle/) when ref_kat is not built.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8192, help="ciphertexts per GPU")
    ap.add_argument("--params", default="STD128",
                    help="parameter set (default STD128 = the BASELINE metric; e.g. STD192 for the C4 class, "
                         "device-resident, with --no-cpu-baseline)")
    ap.add_argument("--kernel-reps", type=int, default=2, help="blind-rotation launches timed for the roofline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--generic", action="store_true", help="force the generic LDS blind-rotation kernel")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend ('nccl' = RCCL; 'gloo' only to rehearse N ranks on fewer GPUs)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline sample length")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r03_pmc_blind_rotate.json"))
    ap.add_argument("--valu-peak-json", default=os.path.join(ROOT, "profiles", "r03_valu_peak.json"))
    ap.add_argument("--no-host-array", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the reference-through-the-shim leg")
    return ap.parse_args()


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


def host_threads():
    """Threads for the CPU baseline: every core this process may run on, unless the pool caps
    OpenMP (OMP_NUM_THREADS is set to the box's CPU share on the GPU pool)."""
    visible = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(visible, cap) if cap else visible), visible


REF_KAT = os.path.join(ROOT, "oracle", "_ref", "ref_kat")
REF_DROPIN = os.path.join(ROOT, "oracle", "_ref", "ref_dropin")


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


def cpu_baseline_reference(p, seconds, gpu_sample):
    """The reference's own OpenFHE code (oracle/_ref/ref_kat, vector EvalBinGate, CPU functions
    behind the seven GPU symbols, OpenMP over ciphertexts) on K pairs; the first ones are the
    GPU's benchmarked inputs, whose outputs are compared bit for bit."""
    import subprocess
    import tempfile

    threads, visible = host_threads()
    g1, g2, gout = gpu_sample
    per_gate_s = 0.12  # one OpenFHE STD128 gate per thread on the GPU box (profiles/r03z: 800 pairs, 16 threads, 5.9 s)
    K = max(len(g1), int(seconds * threads / per_gate_s))
    rs = np.random.default_rng(5)
    c1 = np.concatenate([g1, rs.integers(0, p.q, (K - len(g1), p.n + 1), dtype=np.uint64)])
    c2 = np.concatenate([g2, rs.integers(0, p.q, (K - len(g2), p.n + 1), dtype=np.uint64)])

    def run(a1, a2, nthreads):
        with tempfile.TemporaryDirectory() as tmp:
            f1, f2, fo = (os.path.join(tmp, x) for x in ("c1", "c2", "out"))
            a1.tofile(f1)
            a2.tofile(f2)
            env = dict(os.environ, OMP_NUM_THREADS=str(nthreads))
            r = subprocess.run([REF_KAT, "ctx=set:STD128", "keys=synth:1", "op=NAND", "api=vector", f"in={f1}",
                                f"in2={f2}", f"out={fo}"], capture_output=True, text=True, env=env, timeout=900)
            if r.returncode:
                raise RuntimeError(r.stderr[-2000:])
            js = json.loads(r.stdout.strip().splitlines()[-1])
            return js, np.fromfile(fo, dtype=np.uint64).reshape(len(a1), p.n + 1)

    js, out = run(c1, c2, threads)
    B1 = max(2, int(seconds / 4 / per_gate_s))
    js1, _ = run(c1[:B1], c2[:B1], 1)
    parity = {"ciphertexts": int(len(gout)), "bit_exact": bool(np.array_equal(out[:len(gout)], gout)),
              "vs": "the reference's OpenFHE CPU path (oracle/_ref/ref_kat), same keys and inputs"}
    return {"value": round(K / js["best_s"], 3), "unit": "bootstraps/s", "cores": threads, "kind": "reference",
            "host_cores_visible": visible, "single_thread_value": round(B1 / js1["best_s"], 3),
            "sample": f"STD128 EvalBinGate(NAND), vector API of the reference's OpenFHE (compiled from its sources, "
                      f"oracle/Makefile.ref) with its CPU accumulator / key switch behind the GPU symbols, OpenMP "
                      f"over ciphertexts, {threads} threads: {K} pairs in {js['best_s']:.1f} s (key load "
                      f"{js['key_load_s']:.1f} s not counted); single thread: {B1} pairs in {js1['best_s']:.1f} s",
            "gpu_parity": parity}


def cpu_baseline(p, bsk, ksk, seconds, gpu_sample=None):
    if os.path.exists(REF_KAT) and gpu_sample is not None:
        try:
            return cpu_baseline_reference(p, seconds, gpu_sample)
        except Exception as e:  # fall back to the restatement
            print(f"[bench] reference CPU baseline failed ({e}); using the C restatement", file=sys.stderr)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    pyoracle.build()
    threads, visible = host_threads()
    orc = pyoracle.Oracle(p_oracle(pyoracle, p), bsk, ksk, threads=threads)
    rs = np.random.default_rng(5)
    # calibrate on one gate per thread, then size the sample to ~`seconds`
    B0 = threads
    c1 = rs.integers(0, p.q, (B0, p.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, p.q, (B0, p.n + 1), dtype=np.uint64)
    t0 = time.perf_counter()
    orc.eval_bin_gate("NAND", c1, c2)
    t_cal = time.perf_counter() - t0
    reps = max(1, int(seconds / max(t_cal, 1e-3)))
    B = B0 * reps
    c1 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    t0 = time.perf_counter()
    orc.eval_bin_gate("NAND", c1, c2)
    dt = time.perf_counter() - t0
    # the single-thread figure SURVEY 8(d) asks for, on a quarter of the time budget
    orc.L.or_set_threads(1)
    B1 = max(1, int(seconds / 4 / max(t_cal, 1e-3)))
    t0 = time.perf_counter()
    orc.eval_bin_gate("NAND", c1[:B1], c2[:B1])
    dt1 = time.perf_counter() - t0
    orc.L.or_set_threads(threads)
    # the same oracle checks the benchmarked GPU outputs (first ciphertexts of the last step)
    parity = None
    if gpu_sample is not None:
        g1, g2, gout = gpu_sample
        ref = orc.eval_bin_gate("NAND", g1, g2)
        parity = {"ciphertexts": int(len(gout)), "bit_exact": bool(np.array_equal(ref, gout)),
                  "vs": "oracle/tfhe_oracle.c on the same synthetic keys and inputs"}
    orc.close()
    return {"value": round(B / dt, 3), "unit": "bootstraps/s", "cores": threads, "kind": "port",
            "host_cores_visible": visible, "single_thread_value": round(B1 / dt1, 3),
            "sample": f"STD128 EvalBinGate(NAND) on {B} random ciphertext pairs, same synthetic keys; "
                      f"oracle/tfhe_oracle.c (exact u128 CPU restatement, OpenMP one ciphertext per thread); "
                      f"{dt:.1f} s; single thread: {B1} pairs in {dt1:.1f} s",
            "gpu_parity": parity}


def p_oracle(pyoracle, p):
    return pyoracle.params_from_set("STD128")


def main():
    args = parse()
    if args.params != "STD128" and not args.no_cpu_baseline:
        sys.exit("[bench] the cpu_baseline leg is defined for STD128; add --no-cpu-baseline")
    if args.generic:
        os.environ["TFHE_FORCE_GENERIC"] = "1"
    import torch
    import torch.distributed as dist
    import tfhe_amd
    from tfhe_amd import dist as tdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    local_dev = local % max(1, torch.cuda.device_count())  # == local on a full node
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    p = tfhe_amd.params_from_set(args.params)
    B = args.batch
    # a dedicated (non-null) stream: the engine's kernels, torch's tensors and the
    # HIP events below are all ordered on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    # ---- GPUSetup: rank 0 converts the keys, the image is broadcast over RCCL ----
    t_setup = time.perf_counter()
    bcast_ms = None
    if rank == 0:
        bsk, ksk = synthetic_keys(p)
        ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
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
            ctx = tfhe_amd.BinFHEContextHIP.from_key_image(p, img.data_ptr(), img.numel(), local_dev)
        del img
    setup_s = time.perf_counter() - t_setup

    # ---- inputs resident in HBM ----
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    ct1 = torch.randint(0, int(p.q), (B, p.n + 1), dtype=torch.int64, device=dev, generator=g)
    ct2 = torch.randint(0, int(p.q), (B, p.n + 1), dtype=torch.int64, device=dev, generator=g)
    out = torch.empty((B, p.n + 1), dtype=torch.int64, device=dev)

    def step():
        ctx.EvalBinGateDevice("NAND", B, ct1.data_ptr(), ct2.data_ptr(), out.data_ptr(), stream=sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
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
    total_bs = B * args.steps * world
    value = total_bs / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- dominant kernel (blind rotation) timed alone with HIP events on its stream ----
    a = ct1[:, : p.n].contiguous()
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
    balg, bsk_bytes = b_alg_per_bootstrap(p)
    traffic, valu_insts, pmc = None, None, {}
    if os.path.exists(args.pmc_json):
        try:
            pmc = json.load(open(args.pmc_json))
            if pmc.get("units_per_launch") == B:
                traffic = pmc.get("hbm_bytes_per_launch")
                valu_insts = pmc.get("sq_insts_valu_per_launch")
            else:
                pmc = {}
        except Exception:
            traffic, valu_insts, pmc = None, None, {}
    mm = modmuls_per_bootstrap(p)
    achieved_mm = mm * B / (br_ms * 1e-3)
    peak_mm, peak_src = None, None
    if os.path.exists(args.valu_peak_json):
        vp = json.load(open(args.valu_peak_json))
        peak_mm, peak_src = vp["modmul_per_s"], vp
    roofline = {"bound": "valu-int", "achieved": round(achieved_mm / 1e12, 3),
                "peak": None if peak_mm is None else round(peak_mm / 1e12, 3), "unit": "Tmodmul/s",
                "frac": None if peak_mm is None else round(achieved_mm / peak_mm, 3), "traffic": traffic,
                "kernel": "blind_rotate (tfhe_eval_acc_device)", "kernel_ms": round(br_ms, 3),
                "units_per_launch": B, "alg_modmul_per_unit": mm,
                "hbm_frac": None if traffic is None else round(traffic / (br_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4),
                "effective_keystream_tbs": round(balg * B / (br_ms * 1e-3) / 1e12, 2), "alg_bytes_per_unit": balg,
                "note": "achieved = SURVEY 8(d) algorithmic modmuls per bootstrap x batch / event-timed kernel; peak = "
                        "signed-Montgomery modmul rate of the VALU microbenchmark "
                        + ("(" + os.path.relpath(args.valu_peak_json, ROOT) + ", " + str(peak_src.get("clock", "")) + ")"
                           if peak_src else "(not found)")
                        + "; hbm_frac = PMC HBM bytes / kernel time / 8 TB/s; effective_keystream_tbs = B_alg "
                          "(no cross-ciphertext reuse) x batch / kernel time, served from L2/MALL"}
    simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
    valu = {"bound": "valu-int", "modmul_per_bootstrap": mm,
            "achieved_modmul_per_s": round(mm * B / (br_ms * 1e-3), 1),
            "valu_instr_per_launch": valu_insts,
            "issue_frac": None if valu_insts is None else
            round(valu_insts * VALU_CYCLES / (simds * CLOCK_HZ * br_ms * 1e-3), 3),
            "note": "issue_frac = PMC SQ_INSTS_VALU x 4 cycles / (4 SIMDs/CU x CUs x 2.4 GHz x kernel time), "
                    "from " + os.path.relpath(args.pmc_json, ROOT)}
    act, gui = pmc.get("sq_active_inst_valu_per_launch"), pmc.get("grbm_gui_active_per_launch")
    if act and gui:
        # measured in one PMC pass, clock-independent: VALU-executing cycles per SIMD over the
        # launch's cycles (GRBM_GUI_ACTIVE sums the 8 XCDs; SQ_ACTIVE_INST_VALU is quad-cycles)
        valu["busy_frac"] = round(act * 4 / simds / (gui / 8), 3)
        pass_ns = pmc.get("gui_pass_kernel_ns_per_launch")  # the GUI pass's own dispatch time
        valu["held_clock_ghz"] = round(gui / 8 / (pass_ns * 1e-9 if pass_ns else br_ms * 1e-3) / 1e9, 2)
        valu["note"] += ("; busy_frac = SQ_ACTIVE_INST_VALU x 4 / SIMDs / (GRBM_GUI_ACTIVE / 8); held_clock_ghz = "
                         "GRBM_GUI_ACTIVE / 8 / kernel time (profiled pass, MI355X_MICROARCH.md 'DVFS give-back')")
        if peak_mm and peak_src.get("held_clock_ghz"):
            # the same peak scaled to the clock the part holds under this kernel (power-limited): how much
            # of the gap is issue efficiency and how much is clock
            peak_k = peak_mm * valu["held_clock_ghz"] / peak_src["held_clock_ghz"]
            roofline["frac_at_kernel_clock"] = round(achieved_mm / peak_k, 3)
            roofline["note"] += (f"; frac_at_kernel_clock = achieved / (peak x {valu['held_clock_ghz']} GHz held under "
                                 f"the kernel / {peak_src['held_clock_ghz']} GHz held under the microbenchmark)")

    # ---- the same gates through the host-array entry point (PCIe + host staging included) ----
    host_array = None
    if rank == 0 and world == 1 and not args.no_host_array:
        h1 = ct1.cpu().numpy().astype(np.uint64)
        h2 = ct2.cpu().numpy().astype(np.uint64)
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            hout = ctx.EvalBinGate("NAND", h1, h2)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        host_array = {"value": round(B / best, 1), "unit": "bootstraps/s", "ms": round(best * 1e3, 3),
                      "equal_to_device_resident": bool(np.array_equal(hout, out.cpu().numpy().astype(np.uint64))),
                      "note": "tfhe_eval_bin_gate on host arrays: H2D + kernels + D2H through pinned staging, best of 2"}

    dropin = None
    if rank == 0 and world == 1 and args.params == "STD128" and not args.no_dropin and host_array is not None:
        try:
            dropin = dropin_leg(h1, h2, out.cpu().numpy().astype(np.uint64), host_array["ms"])
        except Exception as e:  # reported, never fatal: the headline does not depend on it
            print(f"[bench] drop-in leg failed: {e}", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if bsk is None:
            bsk, ksk = synthetic_keys(p)
        K = min(B, 64)
        sample = tuple(x[:K].cpu().numpy().astype(np.uint64) for x in (ct1, ct2, out))
        cpu = cpu_baseline(p, bsk, ksk, args.cpu_seconds, sample)
        if cpu["gpu_parity"] and not cpu["gpu_parity"]["bit_exact"]:
            print("[bench] ERROR: GPU outputs differ from the CPU reference", file=sys.stderr)

    if rank == 0:
        line = {
            "metric": f"bootstraps/sec (whole node), {args.params} GINX batch={B}",
            "value": round(value, 2), "unit": "bootstraps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "data": "synthetic",
            "dtype": {0: "u32" if int(ctx.info().word_bits) == 32 else "u64", 1: "u32", 2: "f64",
                      3: "f64", 4: "i32", 5: "u64"}[int(ctx.info().br_kernel)],
            "config": {"workload": f"{args.params} GINX EvalBinGate(NAND), inputs resident in HBM",
                       "global_batch": B * world, "batch_per_gpu": B, "n": p.n, "N": p.N, "Q": p.Q,
                       "dG2": p.dG2, "parallelism": f"shard{world}"},
            "roofline": roofline, "valu": valu, "host_array": host_array, "dropin": dropin, "cpu_baseline": cpu,
            "setup_s": round(setup_s, 2), "key_broadcast_ms": None if bcast_ms is None else round(bcast_ms, 2),
            "key_image_bytes": int(ctx.info().key_image_bytes),
        }
        print(json.dumps(line), flush=True)
    ctx.GPUClean()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
