#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output for one kernel into per-launch HBM bytes.

Usage: pmc_summary.py KERNEL_SUBSTRING FETCH_DIR WRITE_DIR OUT_JSON [MIX_DIR ...]
MIX_DIR... (optional): passes with SQ_INSTS_VALU / SQ_INSTS_LDS / SQ_WAVES and SQ_ACTIVE_INST_VALU /
GRBM_GUI_ACTIVE, recorded per launch (bench.py turns them into the VALU issue fraction, the measured
VALU-busy fraction and the clock the chip held).
FETCH_SIZE/WRITE_SIZE are KiB (TCC_EA0_RDREQ/WRREQ based).  Per
MI355X_MICROARCH.md 'HBM', gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide
(16 B/lane) coalesced stream; other access widths are uncalibrated, so both the
raw and the x2-corrected read figures are recorded.
"""
import csv
import glob
import json
import os
import sys


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def per_launch(rs, kname, counter):
    vals = [float(r["Counter_Value"]) for r in rs if kname in r.get("Kernel_Name", "") and r["Counter_Name"] == counter]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    kname, fdir, wdir, out = sys.argv[1:5]
    fetch, nf = per_launch(rows(fdir), kname, "FETCH_SIZE")
    write, nw = per_launch(rows(wdir), kname, "WRITE_SIZE")
    res = {"kernel": kname, "launches": [nf, nw], "fetch_kib_raw": fetch, "write_kib": write,
           "units_per_launch": int(os.environ.get("PMC_UNITS", "8192"))}  # bench.py's default batch
    if fetch is not None and write is not None:
        res["hbm_bytes_per_launch_raw"] = (fetch + write) * 1024
        res["hbm_bytes_per_launch"] = (2 * fetch + write) * 1024
        res["correction"] = "read side x2 per MI355X_MICROARCH.md HBM section (wide-stream calibration)"
    for d in sys.argv[5:]:
        mix = rows(d)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_VALU",
                  "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
            v, _ = per_launch(mix, kname, c)
            if v is not None:
                res[c.lower() + "_per_launch"] = v
        # duration of the profiled dispatches that carried GRBM_GUI_ACTIVE (same pass: clock = GUI / 8 / time)
        ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in mix
              if kname in r.get("Kernel_Name", "") and r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("End_Timestamp")]
        if ds:
            res["gui_pass_kernel_ns_per_launch"] = sum(ds) / len(ds)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
