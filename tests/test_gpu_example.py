"""Runs examples/time_estimate (built by __graft_entry__.build() / examples/Makefile) on the GPU:
the five operations of the reference's time-estimate.cpp through the C-ABI from a C++ caller.
Values are synthetic (no decryption); the parity of each entry point is tests/test_gpu_parity.py's."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_time_estimate_example_runs():
    exe = os.path.join(ROOT, "examples", "time_estimate")
    assert os.path.exists(exe), "examples/time_estimate not built (run __graft_entry__.build())"
    r = subprocess.run([exe, "256"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    print(r.stdout)
    ops = re.findall(r"^(\w+)\s+batch\s+256\s+([0-9.]+) ms / ctx", r.stdout, re.M)
    assert [o for o, _ in ops] == ["EvalBinGate", "EvalFunc", "EvalFloor", "EvalSign", "EvalDecomp"]
    assert all(float(ms) > 0 for _, ms in ops)
