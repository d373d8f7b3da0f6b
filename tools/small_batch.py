#!/usr/bin/env python3
"""Small-batch behaviour on one MI355X (VERDICT r3 "next" 2 and 5).

  sign   EvalSign on the C5 contexts (C5a STD128Q, C5b STD128 logQ = 23 throw = 1), ciphertext
         modulus 2^23, device-resident, at B = 128 / 256 / 512 / 1024 -- 128 is the per-GPU shard
         of C5's 1024 on 8 GPUs -- plus the blind rotation alone at the same B; per-ciphertext
         rate relative to B = 1024.  The first 4 outputs of every size are checked bit for bit
         against the oracle (same keys and inputs).
  and    the reference's CHES-experiments.cpp:30-61: STD128 AND on 256 pairs, 1000 calls
         (host-array API and device-resident), and the same through the unchanged reference
         code on the shim (oracle/_ref/ref_dropin) when present.
  split  STD128 NAND and its blind rotation at B = 64 .. 2048, fast4's two-group form against the
         one-group kernel (the tfhe_knobs.split4 threshold)
  func   CHES-experiments.cpp:64-126: EvalFunc(x^3 mod p) in GenerateBinFHEContext(STD128, true,
         12, 0, GINX, false, 1 << 18) at B = 1, 8, 64, 256, 512 (host-array, device-resident, and
         the drop-in through ref_dropin sizes=...).
  arb    C3's context (arbFunc logQ 12, one transformed digit): EvalFunc(m^3 mod 8) and the blind rotation
         at B = 64 .. 4096, the two-workgroup sfduo<1> against the one-workgroup sf2<1> at the duo batches.
  duo2   C5b's context at 128: sfduo<2> (the default) against sf2duo (test library, probe 13) and one workgroup.

    python3 tools/small_batch.py [sign] [and] [func] [split] [arb] [duo2] [--reps 5]

One JSON line per measurement.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-gpu_amd"), os.path.join(ROOT, "oracle")]
DROPIN = os.path.join(ROOT, "oracle", "_ref", "ref_dropin")


def emit(d):
    print(json.dumps(d), flush=True)


def progress(msg):  # keeps the log growing during long key setups
    print(f"[small_batch {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def timed(fn, reps, sync):
    fn()
    sync()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        sync()
        ts.append(time.perf_counter() - t0)
    return min(ts), sum(ts) / len(ts)


def run_sign(reps):
    import torch

    import pyoracle
    import tfhe_amd
    from bench import SIGN_MOD, synthetic_keys

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    sync = lambda: torch.cuda.synchronize(dev)
    for name, p, po in (("C5a", tfhe_amd.params_from_set("STD128Q"), pyoracle.params_from_set("STD128Q")),
                        ("C5b", tfhe_amd.params_from_logq("STD128", False, 23, 0, 0, 1),
                         pyoracle.params_from_logq("STD128", False, 23, 0, 0, 1))):
        progress(f"{name}: keys")
        bsk, ksk = synthetic_keys(p)
        ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
        progress(f"{name}: oracle")
        orc = pyoracle.Oracle(po, bsk, ksk)
        del bsk, ksk
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        full = torch.randint(0, SIGN_MOD, (1024, p.n + 1), dtype=torch.int64, device=dev, generator=g)
        rows = []
        for B in (128, 256, 512, 1024):
            progress(f"{name}: B={B}")
            ct = full[:B].contiguous()
            out = torch.empty_like(ct)
            b0 = ctx.info().bootstraps
            ctx.EvalSignDevice(B, ct.data_ptr(), SIGN_MOD, out.data_ptr(), stream=sp)
            sync()
            per = (ctx.info().bootstraps - b0) // B
            best, mean = timed(lambda: ctx.EvalSignDevice(B, ct.data_ptr(), SIGN_MOD, out.data_ptr(), stream=sp),
                               reps, sync)
            a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
            acc = torch.zeros((B, 2, p.N), dtype=torch.int64, device=dev)
            lib = tfhe_amd.lib()
            br, _ = timed(lambda: tfhe_amd.capi.check(
                lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp), "eval_acc"),
                reps, sync)
            k = 4
            h = ct[:k].cpu().numpy().astype(np.uint64)
            exact = bool(np.array_equal(out[:k].cpu().numpy().astype(np.uint64), orc.eval_sign(h, SIGN_MOD)))
            row = {"B": B, "ms_per_call": round(best * 1e3, 3), "mean_ms": round(mean * 1e3, 3),
                   "bootstraps_per_ct": per, "bootstraps_per_s": round(B * per / best, 1),
                   "blind_rotation_ms": round(br * 1e3, 3), "parity_4": exact}
            if B <= ctx.knobs()["duo"]:  # the same call on the one-workgroup form (A/B, same box)
                with ctx.knobs_set(duo=0):
                    b1, _ = timed(lambda: ctx.EvalSignDevice(B, ct.data_ptr(), SIGN_MOD, out.data_ptr(), stream=sp),
                                  reps, sync)
                    br1, _ = timed(lambda: tfhe_amd.capi.check(
                        lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp),
                        "eval_acc"), reps, sync)
                    one = out[:k].cpu().numpy().astype(np.uint64)
                ctx.EvalSignDevice(B, ct.data_ptr(), SIGN_MOD, out.data_ptr(), stream=sp)
                sync()
                row.update(one_workgroup_ms_per_call=round(b1 * 1e3, 3), one_workgroup_blind_rotation_ms=round(br1 * 1e3, 3),
                           two_equal_one=bool(np.array_equal(one, out[:k].cpu().numpy().astype(np.uint64))))
            rows.append(row)
        ref = rows[-1]["bootstraps_per_s"]
        for r in rows:
            r["rate_vs_1024"] = round(r["bootstraps_per_s"] / ref, 3)
        emit({"what": f"{name} EvalSign (modulus 2^23) device-resident batch sweep", "kernel": int(ctx.info().br_kernel),
              "rows": rows})
        orc.close()
        ctx.GPUClean()


def run_and(reps_calls=1000):
    import torch

    import tfhe_amd
    from bench import synthetic_keys

    p = tfhe_amd.params_from_set("STD128")
    bsk, ksk = synthetic_keys(p)
    ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
    rs = np.random.default_rng(3)
    B = 256
    c1 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, p.q, (B, p.n + 1), dtype=np.uint64)
    ctx.EvalBinGate("AND", c1, c2)
    t0 = time.perf_counter()
    for _ in range(reps_calls):
        ho = ctx.EvalBinGate("AND", c1, c2)
    host_s = time.perf_counter() - t0
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    d1 = torch.from_numpy(c1.astype(np.int64)).to(dev)
    d2 = torch.from_numpy(c2.astype(np.int64)).to(dev)
    do = torch.empty_like(d1)
    ctx.EvalBinGateDevice("AND", B, d1.data_ptr(), d2.data_ptr(), do.data_ptr(), stream=sp)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps_calls):
        ctx.EvalBinGateDevice("AND", B, d1.data_ptr(), d2.data_ptr(), do.data_ptr(), stream=sp)
    torch.cuda.synchronize(dev)
    dev_s = time.perf_counter() - t0
    same = bool(np.array_equal(do.cpu().numpy().astype(np.uint64), ho))
    with ctx.knobs_set(split4=0):  # the one-group kernel, same box (A/B)
        ctx.EvalBinGateDevice("AND", B, d1.data_ptr(), d2.data_ptr(), do.data_ptr(), stream=sp)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps_calls):
            ctx.EvalBinGateDevice("AND", B, d1.data_ptr(), d2.data_ptr(), do.data_ptr(), stream=sp)
        torch.cuda.synchronize(dev)
        one_s = time.perf_counter() - t0
        same = same and bool(np.array_equal(do.cpu().numpy().astype(np.uint64), ho))
    res = {"what": "CHES-experiments.cpp:30-61: STD128 AND, 256 pairs, 1000 calls", "B": B, "calls": reps_calls,
           "host_array_total_s": round(host_s, 3), "host_array_ms_per_call": round(host_s / reps_calls * 1e3, 3),
           "device_resident_ms_per_call": round(dev_s / reps_calls * 1e3, 3),
           "device_resident_one_group_ms_per_call": round(one_s / reps_calls * 1e3, 3),
           "host_array_bootstraps_per_s": round(B * reps_calls / host_s, 1), "outputs_equal": same}
    ctx.GPUClean()
    if os.path.exists(DROPIN):
        with tempfile.TemporaryDirectory() as tmp:
            f1, f2 = os.path.join(tmp, "c1"), os.path.join(tmp, "c2")
            c1.tofile(f1)
            c2.tofile(f2)
            r = subprocess.run([DROPIN, "ctx=set:STD128", "keys=synth:1", "op=AND", "api=vector", "gpus=1",
                                f"in={f1}", f"in2={f2}", "reps=50"], capture_output=True, text=True, timeout=600)
            if r.returncode == 0:
                js = json.loads(r.stdout.strip().splitlines()[-1])
                res["dropin_ms_per_call"] = round(js["mean_s"] * 1e3, 3)
                res["dropin_best_ms"] = round(js["best_s"] * 1e3, 3)
            else:
                res["dropin_error"] = r.stderr[-500:]
    emit(res)


def run_split(reps):
    """STD128 NAND device-resident and the blind rotation alone, two-group form (split4 forced on) against the
    one-group kernel (split4 = 0) at batch sizes around the default limit: picks tfhe_knobs.split4."""
    import torch

    import tfhe_amd
    from bench import synthetic_keys

    p = tfhe_amd.params_from_set("STD128")
    bsk, ksk = synthetic_keys(p)
    ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    sync = lambda: torch.cuda.synchronize(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    lib = tfhe_amd.lib()
    rows = []
    for B in (64, 128, 256, 384, 512, 768, 1024, 2048):
        c1 = torch.randint(0, int(p.q), (B, p.n + 1), dtype=torch.int64, device=dev, generator=g)
        c2 = torch.randint(0, int(p.q), (B, p.n + 1), dtype=torch.int64, device=dev, generator=g)
        out = torch.empty_like(c1)
        a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
        acc = torch.zeros((B, 2, p.N), dtype=torch.int64, device=dev)
        row = {"B": B}
        outs = []
        for tag, lim in (("split", 1 << 20), ("one_group", 0)):
            with ctx.knobs_set(split4=lim):
                gate, _ = timed(lambda: ctx.EvalBinGateDevice("NAND", B, c1.data_ptr(), c2.data_ptr(), out.data_ptr(),
                                                              stream=sp), reps, sync)
                outs.append(out.cpu().numpy())
                br, _ = timed(lambda: tfhe_amd.capi.check(
                    lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp), "eval_acc"),
                    reps, sync)
            row[f"{tag}_gate_ms"] = round(gate * 1e3, 3)
            row[f"{tag}_blind_rotation_ms"] = round(br * 1e3, 3)
        row["equal"] = bool(np.array_equal(outs[0], outs[1]))
        rows.append(row)
        progress(f"split B={B}: {row}")
    emit({"what": "STD128 NAND device-resident: two-group fast4 (SPLIT) vs one group", "rows": rows})
    ctx.GPUClean()


def run_func(reps):
    import torch

    import pyoracle
    import tfhe_amd
    from bench import cube_lut, synthetic_keys

    spec = ("STD128", True, 12, 0, 1 << 18, 0)
    p = tfhe_amd.params_from_logq(*spec)
    bsk, ksk = synthetic_keys(p)
    ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
    orc = pyoracle.Oracle(pyoracle.params_from_logq(*spec), bsk, ksk)
    del bsk, ksk
    lut = cube_lut(int(p.q))
    rs = np.random.default_rng(4)
    sizes = (1, 8, 64, 256, 512)
    allct = rs.integers(0, p.q, (max(sizes), p.n + 1), dtype=np.uint64)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    sp = s.cuda_stream
    dl = torch.from_numpy(lut.astype(np.int64)).to(dev)
    rows = []
    for B in sizes:
        progress(f"func B={B}")
        h = allct[:B]
        hb, hm = timed(lambda: ctx.EvalFunc(h, lut), reps, lambda: None)
        ho = ctx.EvalFunc(h, lut)
        d = torch.from_numpy(h.astype(np.int64)).to(dev)
        do = torch.empty_like(d)
        db, dm = timed(lambda: ctx.EvalFuncDevice(B, d.data_ptr(), dl.data_ptr(), do.data_ptr(), stream=sp), reps,
                       lambda: torch.cuda.synchronize(dev))
        k = min(B, 2)
        rows.append({"B": B, "host_array_ms": round(hm * 1e3, 3), "host_array_best_ms": round(hb * 1e3, 3),
                     "device_resident_ms": round(dm * 1e3, 3), "device_resident_best_ms": round(db * 1e3, 3),
                     "host_eq_device": bool(np.array_equal(ho, do.cpu().numpy().astype(np.uint64))),
                     "parity": bool(np.array_equal(ho[:k], orc.eval_func(h[:k], lut)))})
    orc.close()
    ctx.GPUClean()
    res = {"what": "CHES-experiments.cpp:64-126: EvalFunc(x^3 mod 8), GenerateBinFHEContext(STD128, true, 12, 0, "
                   "GINX, false, 1 << 18); ms per call, mean of the reps", "reps": reps, "rows": rows}
    if os.path.exists(DROPIN):
        progress("func: drop-in sweep (reference key load first)")
        with tempfile.TemporaryDirectory() as tmp:
            fi, fl = os.path.join(tmp, "c"), os.path.join(tmp, "lut")
            allct.tofile(fi)
            lut.tofile(fl)
            r = subprocess.run([DROPIN, "ctx=logq:STD128,1,12,0,262144,0", "keys=synth:1", "op=func", "api=vector",
                                "gpus=1", f"in={fi}", f"lut={fl}", f"mod={p.q}", f"reps={reps}",
                                "sizes=" + ",".join(map(str, sizes))], capture_output=True, text=True, timeout=1200)
            if r.returncode == 0:
                js = json.loads(r.stdout.strip().splitlines()[-1])
                res["dropin"] = [{"B": x["B"], "ms": round(x["mean_s"] * 1e3, 3), "best_ms": round(x["best_s"] * 1e3, 3)}
                                 for x in js["sweep"]]
            else:
                res["dropin_error"] = r.stderr[-500:]
    emit(res)


def run_arb(reps):
    """C3's context (arbFunc logQ 12, one transformed digit) at small batches: EvalFunc(m^3 mod 8) device-resident
    and the blind rotation alone at B = 64 .. 4096; at the duo batches also the one-workgroup sf2<1> (duo = 0) on
    the same box, alternating, and the first 4 outputs against the oracle."""
    import torch

    import pyoracle
    import tfhe_amd
    from bench import cube_lut, synthetic_keys

    spec = ("STD128", True, 12, 0, 0, 1)
    p, po = tfhe_amd.params_from_logq(*spec), pyoracle.params_from_logq(*spec)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    sync = lambda: torch.cuda.synchronize(dev)
    progress("C3: keys")
    bsk, ksk = synthetic_keys(p)
    ctx = tfhe_amd.BinFHEContextHIP(p).GPUSetup(bsk, ksk)
    progress("C3: oracle")
    orc = pyoracle.Oracle(po, bsk, ksk)
    del bsk, ksk
    lut = cube_lut(int(p.q))
    dl = torch.from_numpy(lut.astype(np.int64)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    full = torch.randint(0, int(p.q), (4096, p.n + 1), dtype=torch.int64, device=dev, generator=g)
    lib = tfhe_amd.lib()
    rows = []
    for B in (64, 128, 256, 512, 1024, 4096):
        progress(f"C3: B={B}")
        ct = full[:B].contiguous()
        out = torch.empty_like(ct)
        call = lambda: ctx.EvalFuncDevice(B, ct.data_ptr(), dl.data_ptr(), out.data_ptr(), stream=sp)
        a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
        acc = torch.zeros((B, 2, p.N), dtype=torch.int64, device=dev)
        br_call = lambda: tfhe_amd.capi.check(
            lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp), "eval_acc")
        b0 = ctx.info().bootstraps
        call()
        sync()
        per = (ctx.info().bootstraps - b0) // B
        forms = [("", {})] + ([("one_workgroup_", {"duo": 0})] if B <= ctx.knobs()["duo"] else [])
        res = {k: [[], []] for k, _ in forms}
        for _ in range(2):  # two alternating reps of every form
            for k, kn in forms:
                with ctx.knobs_set(**kn):
                    res[k][0].append(timed(call, reps, sync)[0])
                    res[k][1].append(timed(br_call, reps, sync)[0])
        call()
        sync()
        h = ct[:4].cpu().numpy().astype(np.uint64)
        exact = bool(np.array_equal(out[:4].cpu().numpy().astype(np.uint64), orc.eval_func(h, lut)))
        best = min(res[""][0])
        row = {"B": B, "ms_per_call": round(best * 1e3, 3), "bootstraps_per_ct": per,
               "bootstraps_per_s": round(B * per / best, 1), "blind_rotation_ms": round(min(res[""][1]) * 1e3, 3),
               "parity_4": exact}
        if len(forms) > 1:
            row.update(one_workgroup_ms_per_call=round(min(res["one_workgroup_"][0]) * 1e3, 3),
                       one_workgroup_blind_rotation_ms=round(min(res["one_workgroup_"][1]) * 1e3, 3))
        rows.append(row)
    ref = rows[-1]["bootstraps_per_s"]
    for r in rows:
        r["rate_vs_4096"] = round(r["bootstraps_per_s"] / ref, 3)
    emit({"what": "C3 arbFunc logQ 12 EvalFunc(m^3 mod 8) device-resident batch sweep",
          "kernel": int(ctx.info().br_kernel), "duo_timeouts": int(ctx.info().duo_timeouts), "rows": rows})
    orc.close()
    ctx.GPUClean()


def run_duo2(reps, libpath=None):
    """C5b's context (two transformed digits) at the 8-GPU shard (128): the blind rotation and EvalSign on
    sfduo<2> (split by NTT half, the default since round 6), on sf2duo (split by accumulator polynomial; test
    library, probe 13) and on one workgroup per ciphertext, alternating on one box; outputs compared.
    (profiles/r06l, r06m: run before the default changed, so their "sf2duo" key is the default form of then,
    sf2duo, and "sfduo2" is probe 13 of then, sfduo<2>.)"""
    import torch

    import tfhe_amd
    from bench import SIGN_MOD, synthetic_keys

    p = tfhe_amd.params_from_logq("STD128", False, 23, 0, 0, 1)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    sync = lambda: torch.cuda.synchronize(dev)
    progress("C5b: keys")
    bsk, ksk = synthetic_keys(p)
    ctx = tfhe_amd.BinFHEContextHIP(p, library=libpath or tfhe_amd.capi.TEST_LIB).GPUSetup(bsk, ksk)
    del bsk, ksk
    lib = ctx._L  # the test library the context was set up on
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    B = 128
    ct = torch.randint(0, SIGN_MOD, (B, p.n + 1), dtype=torch.int64, device=dev, generator=g)
    out = torch.empty_like(ct)
    a = torch.randint(0, int(p.q), (B, p.n), dtype=torch.int64, device=dev, generator=g)
    acc0 = torch.randint(0, int(p.Q), (B, 2, p.N), dtype=torch.int64, device=dev, generator=g)
    acc = acc0.clone()
    sign = lambda: ctx.EvalSignDevice(B, ct.data_ptr(), SIGN_MOD, out.data_ptr(), stream=sp)
    br = lambda: tfhe_amd.capi.check(lib.tfhe_eval_acc_device(ctx.handle, B, a.data_ptr(), int(p.q), acc.data_ptr(), sp),
                                     "eval_acc")
    forms = [("sfduo2", {}), ("sf2duo", {"probe": 13}), ("one_workgroup", {"duo": 0})]
    res = {k: {"sign_ms": [], "br_ms": []} for k, _ in forms}
    outs = {}
    for _ in range(3):
        for k, kn in forms:
            with ctx.knobs_set(**kn):
                progress(f"C5b 128: {k}")
                res[k]["sign_ms"].append(round(timed(sign, reps, sync)[0] * 1e3, 3))
                res[k]["br_ms"].append(round(timed(br, reps, sync)[0] * 1e3, 3))
                acc.copy_(acc0)
                br()
                sign()
                sync()
                outs[k] = (acc.cpu().numpy(), out.cpu().numpy())
    same = all(np.array_equal(outs[k][0], outs["one_workgroup"][0]) and np.array_equal(outs[k][1], outs["one_workgroup"][1])
               for k in outs)
    emit({"what": "C5b at 128: sf2duo vs sfduo<2> vs one workgroup (alternating, one box)", "B": B, "lib": libpath,
          "forms": res, "outputs_equal": same, "duo_timeouts": int(ctx.info().duo_timeouts)})
    ctx.GPUClean()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="*", default=["sign", "and", "func"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None, help="duo2: a test-library build (default lib/libtfhe_hip_test.so)")
    args = ap.parse_args()
    for w in args.what:
        {"sign": lambda: run_sign(args.reps), "and": lambda: run_and(), "func": lambda: run_func(args.reps),
         "split": lambda: run_split(args.reps), "arb": lambda: run_arb(args.reps),
         "duo2": lambda: run_duo2(args.reps, args.lib)}[w]()


if __name__ == "__main__":
    main()
