"""The round-0 race of the wave-local N = 2048 FP64 kernel (k_blind_rotate_f64w), reproduced
deterministically and shown fixed.

The kernel's prologue transforms the folded accumulator C' (passes B, C and the units run
wave-local, each wave on its own 256-entry block of the LDS buffer), and round 0's first pass A
writes every block.  Round 2 had no barrier between the two: a wave that left the prologue first
overwrote blocks that slower waves were still reading, and whole STD128Q / STD192 ciphertexts came
out wrong on some runs.  The fault probe (the probe knob; its kernel builds exist only
in the test library lib/libtfhe_hip_test.so, blind_rotate_f64.hip under -DTFHE_TEST_PROBES) makes the
timing deterministic: waves 1.. sleep inside the prologue transform, so wave 0 always reaches round 0
first.  With the barrier (probe 2) results stay bit-exact to the oracle; without it (probe 3, the
round-2 kernel) they do not.  The product library refuses the probe knob.
"""
import numpy as np
import pytest

import tfhe_amd

pytestmark = pytest.mark.gpu

B = 4


@pytest.fixture(scope="module")
def std128q(oracle):
    op, cp = oracle.params_from_set("STD128Q"), tfhe_amd.params_from_set("STD128Q")
    rs = np.random.default_rng(23)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx = tfhe_amd.BinFHEContextHIP(cp, library=tfhe_amd.capi.TEST_LIB).GPUSetup(bsk, ksk)
    orc = oracle.Oracle(op, bsk, ksk)
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    want = orc.eval_acc(a, op.q, acc)
    yield ctx, op, a, acc, want
    ctx.GPUClean()
    orc.close()


def test_f64w_is_the_kernel(std128q):
    ctx, *_ = std128q
    assert ctx.info().br_kernel == 3  # TFHE_BR_F64_FOLD


def test_repeated_calls_bit_exact(std128q):
    ctx, op, a, acc, want = std128q
    for _ in range(12):
        assert np.array_equal(ctx.EvalAcc(a, op.q, acc), want)


def test_delayed_waves_with_barrier_bit_exact(std128q):
    ctx, op, a, acc, want = std128q
    with ctx.knobs_set(probe=2):
        for _ in range(3):
            assert np.array_equal(ctx.EvalAcc(a, op.q, acc), want)


def test_delayed_waves_without_barrier_reproduce_the_race(std128q):
    ctx, op, a, acc, want = std128q
    with ctx.knobs_set(probe=3):
        got = ctx.EvalAcc(a, op.q, acc)
    wrong = [b for b in range(B) if not np.array_equal(got[b], want[b])]
    assert wrong == list(range(B)), wrong
