#!/usr/bin/env python3
"""The roofline peak of the blind-rotation kernels: the modular-multiply rate of gfx950 VALU
(tools/microbench/valu_rates.hip, every CU saturated with independent signed-Montgomery
products -- the arithmetic of blind_rotate_fast4.hip), and the clock the part held under it
(a separate rocprofv3 --pmc GRBM_GUI_ACTIVE pass of the same binary).

    python3 tools/valu_peak.py RATES_LOG [PMC_DIR] > profiles/<round>_valu_peak.json

RATES_LOG: stdout of tools/microbench/valu_rates; PMC_DIR: rocprofv3 -d of
`rocprofv3 --pmc GRBM_GUI_ACTIVE -- tools/microbench/valu_rates` (optional).
"""
import csv
import glob
import json
import os
import re
import sys


def main():
    log = open(sys.argv[1]).read()
    res = {"source": "tools/microbench/valu_rates.hip", "log": os.path.relpath(sys.argv[1])}
    rates = {}
    for m in re.finditer(r"^(\S+)\s+([\d.]+) ms\s+([\d.]+) Glane-ops/s", log, re.M):
        rates[m.group(1)] = {"ms": float(m.group(2)), "per_s": float(m.group(3)) * 1e9}
    sm = rates["modmul_smont_i32"]
    res.update({"kernel": "modmul_smont_i32", "modmul_per_s": sm["per_s"], "ms": sm["ms"],
                "modmul_f64_per_s": rates.get("modmul_f64_centred", {}).get("per_s"),
                "modmul_shoup_u32_per_s": rates.get("modmul_shoup_u32", {}).get("per_s")})
    dev = re.search(r"^device (.*) CUs=(\d+) clock=(\d+) kHz", log, re.M)
    if dev:
        res["cus"] = int(dev.group(2))
        res["nominal_clock_ghz"] = int(dev.group(3)) / 1e6
    if len(sys.argv) > 2:
        rows = []
        for f in glob.glob(os.path.join(sys.argv[2], "**", "*counter_collection.csv"), recursive=True):
            rows += list(csv.DictReader(open(f)))
        # (dispatch time s, clock GHz) per launch; the timed launch is the long one (the 0.06 ms warm-up
        # launch's counter window overhangs its dispatch time, so its quotient reads above 2.4 GHz)
        clk = [((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9,
                float(r["Counter_Value"]) / 8 / ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9) / 1e9)
               for r in rows if "k_modmul_smont" in r.get("Kernel_Name", "") and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
        if clk:
            res["held_clock_ghz"] = round(max(clk)[1], 3)
    res["clock"] = (f"held {res['held_clock_ghz']} GHz (GRBM_GUI_ACTIVE / 8 / dispatch time)" if "held_clock_ghz" in res
                    else "clock not measured")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
