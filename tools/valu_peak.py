#!/usr/bin/env python3
"""The roofline peaks of the blind-rotation kernels: the modular-multiply rate of gfx950 VALU for
each arithmetic the kernels use (tools/microbench/valu_rates.hip, every CU saturated with
independent products), and the clock the part held under each (a separate rocprofv3 --pmc
GRBM_GUI_ACTIVE pass of the same binary).

    python3 tools/valu_peak.py RATES_LOG [PMC_DIR] > profiles/<round>_valu_peak.json

RATES_LOG: stdout of tools/microbench/valu_rates; PMC_DIR: rocprofv3 -d of
`rocprofv3 --pmc GRBM_GUI_ACTIVE -- tools/microbench/valu_rates` (optional).

Peaks by kernel family (bench.py picks the one matching the context's blind rotation):
  smont_i32   signed Montgomery, 3 instructions (blind_rotate_fast4.hip, STD128 class: C2)
  fmod_q37    exact FP64 fmodmul, 6 instructions, Q = 2^37 - 2^17 + 1 (f64w, STD192: C4)
  fmod_q50    the same at Q = 2^50 - 2^14 + 1 (f64w, STD128Q: C5a)
  sf_q54      special-form u64 sf_mul at Q = 2^54 - 77823 (sf2, logQ contexts: C3, C5b)
The fmod and sf kernels call the blind-rotation kernels' own device functions (device_math.hpp).
"""
import csv
import glob
import json
import os
import re
import sys

# (label in the log, substrings of the kernel's name in the rocprofv3 CSV, mangled or not)
FAMILIES = {"smont_i32": ("modmul_smont_i32", ("k_modmul_smont",)),
            "fmod_q37": ("modmul_fmod_q37", ("k_modmul_fmod", "137438822401")),
            "fmod_q50": ("modmul_fmod_q50", ("k_modmul_fmod", "1125899906826241")),
            "sf_q54": ("modmul_sf_q54", ("k_modmul_sf54",))}


def main():
    log = open(sys.argv[1]).read()
    res = {"source": "tools/microbench/valu_rates.hip", "log": os.path.relpath(sys.argv[1])}
    rates = {}
    for m in re.finditer(r"^(\S+)\s+([\d.]+) ms\s+([\d.]+) Glane-ops/s", log, re.M):
        rates[m.group(1)] = {"ms": float(m.group(2)), "per_s": float(m.group(3)) * 1e9}
    sm = rates["modmul_smont_i32"]
    # top-level fields: the headline (smont) peak, as bench.py has read them since round 2
    res.update({"kernel": "modmul_smont_i32", "modmul_per_s": sm["per_s"], "ms": sm["ms"],
                "modmul_f64_per_s": rates.get("modmul_f64_centred", {}).get("per_s"),
                "modmul_shoup_u32_per_s": rates.get("modmul_shoup_u32", {}).get("per_s")})
    dev = re.search(r"^device (.*) CUs=(\d+) clock=(\d+) kHz", log, re.M)
    if dev:
        res["cus"] = int(dev.group(2))
        res["nominal_clock_ghz"] = int(dev.group(3)) / 1e6
    rows = []
    if len(sys.argv) > 2:
        for f in glob.glob(os.path.join(sys.argv[2], "**", "*counter_collection.csv"), recursive=True):
            rows += list(csv.DictReader(open(f)))

    def held(kname):
        # (dispatch time s, clock GHz) per launch; the timed launch is the long one (the 0.06 ms warm-up
        # launch's counter window overhangs its dispatch time, so its quotient reads above 2.4 GHz)
        clk = [((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9,
                float(r["Counter_Value"]) / 8 / ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9) / 1e9)
               for r in rows if all(k in r.get("Kernel_Name", "") for k in kname) and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
        return round(max(clk)[1], 3) if clk else None

    res["peaks"] = {}
    for fam, (label, kname) in FAMILIES.items():
        if label not in rates:
            continue
        res["peaks"][fam] = {"kernel": label, "modmul_per_s": rates[label]["per_s"], "ms": rates[label]["ms"],
                             "held_clock_ghz": held(kname)}
    h = held(("k_modmul_smont",))
    if h is not None:
        res["held_clock_ghz"] = h
    res["clock"] = (f"held {res['held_clock_ghz']} GHz (GRBM_GUI_ACTIVE / 8 / dispatch time)" if "held_clock_ghz" in res
                    else "clock not measured")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
