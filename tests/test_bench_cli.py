"""bench.py's launch contract on the CPU: a run whose process count differs from --gpus fails with
exit status 2 before touching a GPU (the driver's 8-GPU run can then never report a 1-rank number as
an 8-GPU one), and --help lists the per-configuration options."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

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
    for opt in ("--config", "--batch", "--scaling", "--knob", "--pmc-json", "--test-lib"):
        assert opt in r.stdout


def _bench():
    sys.path.insert(0, ROOT)
    import bench

    return bench


def test_both_readings_of_the_headline():
    """BASELINE's 'STD128 GINX batch=8192 at 1/2/4/8 MI355X' read both ways (verdict r5 item 7): weak =
    8192 per GPU (the default), strong = 8192 in all; the metric string names the global batch."""
    b = _bench()
    cfg = dict(b.CONFIGS["C2"])
    assert cfg["scaling"] == "weak"
    assert b.batch_split(cfg, 8192, 8, 3) == (8192, 65536)
    m = b.metric_name("C2", cfg, 65536, 8192, 8)
    assert m == "bootstraps/sec (whole node), STD128 GINX global batch=65536 (8192 per GPU, weak scaling)"
    cfg["scaling"] = "strong"
    shards = [b.batch_split(cfg, 8192, 8, r) for r in range(8)]
    assert shards == [(1024, 8192)] * 8
    assert [b.batch_split(cfg, 1001, 3, r)[0] for r in range(3)] == [334, 334, 333]
    m = b.metric_name("C2", cfg, 8192, 1024, 8)
    assert m == "bootstraps/sec (whole node), STD128 GINX global batch=8192 (sharded over 8 GPUs, strong scaling)"
    m = b.metric_name("C5a", dict(b.CONFIGS["C5a"]), 1024, 1024, 1)
    assert "global batch=1024 (sharded over 1 GPU, strong scaling)" in m and m.startswith("bootstraps/sec (whole node), C5a")


def test_parity_verdict_fails_on_any_disagreeing_check():
    b = _bench()
    good_oracle = {"ranks_checked": 2, "ranks_passed": 2}
    assert b.parity_verdict(None, None, None, good_oracle) == (True, [])
    cpu_bad = {"gpu_parity": {"bit_exact": False}}
    assert b.parity_verdict(cpu_bad, None, None, good_oracle) == (False, ["cpu_baseline.gpu_parity"])
    ha_bad = {"equal_to_device_resident": False}
    assert b.parity_verdict(None, ha_bad, None, good_oracle)[1] == ["host_array.equal_to_device_resident"]
    assert b.parity_verdict(None, None, ha_bad, good_oracle)[1] == ["dropin.equal_to_device_resident"]
    assert b.parity_verdict(None, None, None, {"ranks_checked": 8, "ranks_passed": 7})[1] == ["oracle_sample"]
    assert b.parity_verdict(None, None, None, None)[0] is False  # a check that did not run is not a pass


def test_oracle_sample_check_catches_one_wrong_word(oracle):
    b = _bench()
    p = oracle.params_from_set("TOY")
    rng = oracle.Rng(3)
    sk, bsk, ksk = oracle.keygen(p, rng)
    orc = oracle.Oracle(p, bsk, ksk, threads=1)
    rs = np.random.default_rng(0)
    ct = rs.integers(0, p.q, (2, p.n + 1), dtype=np.uint64)
    cfg = {"ctx": ("set", "TOY"), "op": "sign"}
    out = orc.eval_sign(ct, b.SIGN_MOD)
    orc.close()
    bad = out.copy()
    bad[0, 0] ^= np.uint64(1)
    rec = b.oracle_sample_check(cfg, bsk, ksk, [[ct, out], [ct, bad]], threads=1)
    assert rec["ranks_checked"] == 2 and rec["per_rank"] == [True, False]


@pytest.mark.gpu
def test_bench_line_passes_its_own_checks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "64", "--steps", "1", "--warmup", "1",
                        "--no-cpu-baseline", "--no-dropin"], capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["parity_ok"] is True and line["oracle_sample"]["ranks_passed"] == 1


@pytest.mark.gpu
def test_bench_strong_scaling_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "96", "--scaling", "strong",
                        "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-dropin", "--no-host-array"],
                       capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["scaling"] == "strong" and line["config"]["global_batch"] == 96 and line["parity_ok"] is True
    assert "global batch=96 (sharded over 1 GPU, strong scaling)" in line["metric"]


@pytest.mark.gpu
def test_bench_exits_nonzero_on_wrong_outputs():
    """A fault injection of the test library (probe 6: f64w flips bit 40 of ciphertext 0's accumulator
    word acc1[0]; duo = 0 keeps this small batch on f64w) makes the benchmarked outputs wrong: the line
    says so and the process fails.  (Probe 3, the prologue race, cannot do it here: the gate pipeline's
    test-vector accumulators have acc0 = 0, and the race only overwrites zeros with zeros.)"""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "C5a", "--batch", "8", "--steps",
                        "1", "--warmup", "1", "--no-cpu-baseline", "--test-lib", "--knob", "probe=6", "--knob", "duo=0"],
                       capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 1, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["parity_ok"] is False and "oracle_sample" in line["parity_failed"]
