"""bench.py's launch contract on the CPU: a run whose process count differs from --gpus fails with
exit status 2 before touching a GPU (the driver's 8-GPU run can then never report a 1-rank number as
an 8-GPU one), and --help lists the per-configuration options."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, world=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    if world is not None:
        env["WORLD_SIZE"] = str(world)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_gpus_without_matching_world_size_exits_2():
    r = _run(["--gpus", "2"])  # WORLD_SIZE unset = 1 process
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=1" in r.stderr


def test_world_size_without_matching_gpus_exits_2():
    r = _run(["--gpus", "1"], world=2)
    assert r.returncode == 2, r.stderr


def test_help_lists_configurations():
    r = _run(["--help"])
    assert r.returncode == 0
    for opt in ("--config", "--batch", "--knob", "--pmc-json", "--test-lib"):
        assert opt in r.stdout
