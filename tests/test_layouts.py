"""CPU checks of the kernels' LDS layouts and transform schedules (no GPU).

The N = 2048 transforms of the exact-FP64 kernel and of the generic u64 kernel gen3 share one
schedule (radix-8 passes over stages 0-2, 3-5, 6-8, two radix-4 units on 9-10) and one XOR
swizzle; tools/lds_layouts_f64.py replays the kernels' thread -> element and twiddle formulas
against the plain stage loops and checks every 64-bit LDS access pattern for bank conflicts.
The four-wavefront STD128 kernel's exchanges are checked by tools/lds_layouts4.py.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_tool(name):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", name)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_f64_gen3_transform_schedule_and_banks():
    out = run_tool("lds_layouts_f64.py")
    assert "index algebra: forward and inverse passes equal the stage loops" in out
    assert out.strip().endswith("OK")


def test_fast4_exchange_layouts():
    out = run_tool("lds_layouts4.py")
    ways = [int(w) for w in re.findall(r"max (\d+)-way", out)]
    assert len(ways) == 8 and max(ways) == 1, out


def test_special_form_kernel_bounds():
    """gen3sf / sf2 (blind_rotate_generic.hip): the register-level sf_mul sequence is exact, its
    quotient fits 32 bits, no value reaches 2^64, offset subtractions stay non-negative, and the
    accumulator update needs one subtraction -- for c = 77823 and the largest admitted c."""
    out = run_tool("bounds_sf.py")
    assert out.strip().endswith("OK"), out


def test_wave_local_transform_schedule():
    """sf2 / f64w: the wave-local N = 2048 passes equal the stage loops, passes B, C and the
    units touch only their wave's block of both polynomials, every b64 access is conflict-free."""
    out = run_tool("lds_layouts_wl.py")
    assert "wave-locality: passes B, C and the units stay in the wave's block" in out
    assert out.strip().endswith("OK"), out


def test_fp64_kernel_bounds():
    """f64w for Q near 2^50 (STD128Q): every sum and fmodmul operand of the forward transform
    (one reduction), products, monomial factors, inverse (passes C and B reduce every output) and
    accumulator update stays below 2^53 in the worst case; the round-2 inverse schedule did not."""
    out = run_tool("bounds_f64.py")
    assert out.strip().endswith("OK"), out
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bounds_f64.py"), "--round2"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "OVER 2^53" in r.stdout, r.stdout


def test_duo_fp64_split_transforms():
    """k_blind_rotate_f64wduo (blind_rotate_f64.hip): the NTT-half split transforms of the two-workgroup
    FP64 kernel equal the stage loops, stay wave-local, and are bank-conflict-free (tools/lds_layouts_duo.py)."""
    out = run_tool("lds_layouts_duo.py")
    assert "OK" in out and "FAILED" not in out
