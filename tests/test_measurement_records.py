"""The measurement records bench.py reads (profiles/r03_valu_peak.json, profiles/r03_pmc_blind_rotate.json)
are reproducible from the raw files committed beside them, and physically plausible: the held clocks
are at most the part's 2.4 GHz, and the roofline fractions they imply are at most 1."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MI355X_MAX_CLOCK_GHZ = 2.4


def test_valu_peak_regenerates_from_raw_files():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "valu_peak.py"),
                          os.path.join(ROOT, "profiles", "r03c", "valu_rates.txt"),
                          os.path.join(ROOT, "profiles", "r03c", "valu_pmc")],
                         capture_output=True, text=True, check=True, cwd=ROOT).stdout
    got = json.loads(out)
    committed = json.load(open(os.path.join(ROOT, "profiles", "r03_valu_peak.json")))
    assert got["modmul_per_s"] == committed["modmul_per_s"]
    assert got["held_clock_ghz"] == committed["held_clock_ghz"]
    assert 1.0 < got["held_clock_ghz"] <= MI355X_MAX_CLOCK_GHZ  # the timed launch, not the warm-up one


def test_pmc_record_is_consistent():
    pmc = json.load(open(os.path.join(ROOT, "profiles", "r03_pmc_blind_rotate.json")))
    assert pmc["units_per_launch"] == 8192
    held = pmc["grbm_gui_active_per_launch"] / 8 / (pmc["gui_pass_kernel_ns_per_launch"] * 1e-9) / 1e9
    assert 1.0 < held <= MI355X_MAX_CLOCK_GHZ
    # VALU-busy fraction of SIMD cycles (bench.py busy_frac) within (0, 1]
    simds = 4 * 256
    busy = pmc["sq_active_inst_valu_per_launch"] * 4 / simds / (pmc["grbm_gui_active_per_launch"] / 8)
    assert 0.5 < busy <= 1.0
    # HBM bytes per launch (read side corrected per MI355X_MICROARCH.md) below 8 TB/s over the launch
    assert pmc["hbm_bytes_per_launch"] / (pmc["gui_pass_kernel_ns_per_launch"] * 1e-9) < 8e12


def test_roofline_fraction_from_records_is_at_most_one():
    peak = json.load(open(os.path.join(ROOT, "profiles", "r03_valu_peak.json")))
    pmc = json.load(open(os.path.join(ROOT, "profiles", "r03_pmc_blind_rotate.json")))
    p = {"n": 512, "N": 1024, "dG2": 8}  # STD128
    mm = p["n"] * ((p["dG2"] + 2) * (p["N"] // 2) * 10 + 4 * p["dG2"] * p["N"] + 4 * p["N"])
    assert mm == 45088768
    kernel_s = pmc["gui_pass_kernel_ns_per_launch"] * 1e-9  # the profiled launch (slowest case)
    achieved = mm * pmc["units_per_launch"] / kernel_s
    assert 0.5 < achieved / peak["modmul_per_s"] <= 1.0
