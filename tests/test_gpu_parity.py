"""GPU parity: the HIP engine, called through the C-ABI, must equal the CPU
oracle bit for bit on the same inputs, and reproduce the reference's own KAT
digests (tests/golden/kat_openfhe.json)."""
import json
import os

import numpy as np
import pytest

from helpers import cube_lut, kat_inputs, random_cts

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kat_openfhe.json")


@pytest.fixture(scope="module")
def capi():
    import tfhe_amd

    return tfhe_amd


def make_pair(capi, oracle, op, cp, bsk, ksk, memo=None):
    """(context, oracle); memo = a case key: the oracle is a MemoOracle (below)."""
    ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    orc = MemoOracle(oracle, op, bsk, ksk, memo) if memo is not None else oracle.Oracle(op, bsk, ksk)
    return ctx, orc


_MEMO = {}


class MemoOracle:
    """The oracle of one case whose kernel-form parametrisations (fast / generic / gen3sf / ...) feed the same
    keys and inputs: its results are memoised by (case, call, input digest), so the CPU restatement runs once
    per case instead of once per kernel form (the GPU suite's time, verdict r5 item 8).  The C oracle context
    (a copy of the keys) is created only when a result is missing."""

    def __init__(self, oracle, op, bsk, ksk, key):
        self._args, self.key, self._o = (oracle, op, bsk, ksk), key, None

    def _call(self, name, *args):
        import hashlib

        h = hashlib.blake2b(digest_size=16)
        for x in args:
            h.update(np.ascontiguousarray(x).tobytes() if isinstance(x, np.ndarray) else repr(x).encode())
        k = (self.key, name, h.hexdigest())
        if k not in _MEMO:
            if self._o is None:
                oracle, op, bsk, ksk = self._args
                self._o = oracle.Oracle(op, bsk, ksk)
            _MEMO[k] = getattr(self._o, name)(*args)
        return _MEMO[k]

    def eval_acc(self, a, amod, acc):
        return self._call("eval_acc", a, amod, acc)

    def eval_floor(self, ct, mod, rb):
        return self._call("eval_floor", ct, mod, rb)

    def close(self):
        if self._o is not None:
            self._o.close()
            self._o = None


# ---------------------------------------------------------------- KATs
@pytest.mark.parametrize("name", ["std128", "std192", "arb12"])
def test_gpu_reproduces_reference_kat(capi, oracle, name):
    gold = json.load(open(GOLDEN))["configs"][name]
    p, bsk, ksk, trials = kat_inputs(oracle, name)
    cp = capi.params_from_set("STD128") if name == "std128" else (
        capi.params_from_set("STD192") if name == "std192" else capi.params_from_logq("STD128", True, 12, 0, 0, 1))
    ctx = capi.BinFHEContextHIP(cp).GPUSetup(bsk, ksk)
    c1 = np.stack([t[0] for t in trials])
    c2 = np.stack([t[1] for t in trials])
    out = ctx.EvalFunc(c1, cube_lut(cp.q)) if name == "arb12" else ctx.EvalBinGate("NAND", c1, c2)
    for r, g in zip(out, gold["trials"]):
        assert [int(x) for x in r[:4]] == g["a0_3"]
        assert int(r[-1]) == g["b"]
        assert f"{oracle.fnv1a64(r):016x}" == g["fnv"]
    ctx.GPUClean()


# ---------------------------------------------------------------- boundary calls
@pytest.fixture(scope="module", params=["fast", "generic"])
def std128(request, capi, oracle):
    """STD128 with valid keys, on the specialised kernel (default) and on the
    generic LDS kernel (TFHE_FORCE_GENERIC=1 at setup)."""
    op = oracle.params_from_set("STD128")
    rng = oracle.Rng(7)
    sk, bsk, ksk = oracle.keygen(op, rng)
    cp = capi.params_from_set("STD128")
    if request.param == "generic":
        os.environ["TFHE_FORCE_GENERIC"] = "1"
    try:
        ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk)
    finally:
        os.environ.pop("TFHE_FORCE_GENERIC", None)
    yield dict(op=op, cp=cp, sk=sk, ctx=ctx, orc=orc, rng=rng, path=request.param)
    ctx.GPUClean()
    orc.close()


def test_eval_acc_parity(std128):
    op, ctx, orc = std128["op"], std128["ctx"], std128["orc"]
    rs = np.random.default_rng(1)
    B = 5
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    acc[0, 0, :] = 0  # a sparse test-vector-like accumulator too
    for amod in (op.q, op.q // 2, 2 * op.N, 4):
        g = ctx.EvalAcc(a % amod, amod, acc)
        c = orc.eval_acc(a % amod, amod, acc)
        assert np.array_equal(g, c), amod


def test_mkm_parity(std128):
    op, ctx, orc = std128["op"], std128["ctx"], std128["orc"]
    rs = np.random.default_rng(2)
    ext = rs.integers(0, op.Q, (33, op.N + 1), dtype=np.uint64)
    ext[0, :] = 0
    ext[1, :] = op.Q - 1
    for fmod in (op.q, 2 * op.q, 1 << 20):
        assert np.array_equal(ctx.MKMSwitch(ext, fmod), orc.mkm_switch(ext, fmod))


# ---------------------------------------------------------------- vector surface
GATES = ["OR", "AND", "NOR", "NAND", "XOR_FAST", "XNOR_FAST", "XOR", "XNOR"]
TRUTH = {"AND": lambda x, y: x & y, "OR": lambda x, y: x | y, "NAND": lambda x, y: 1 - (x & y),
         "NOR": lambda x, y: 1 - (x | y), "XOR": lambda x, y: x ^ y, "XNOR": lambda x, y: 1 - (x ^ y),
         "XOR_FAST": lambda x, y: x ^ y, "XNOR_FAST": lambda x, y: 1 - (x ^ y)}


@pytest.mark.parametrize("gate", GATES)
def test_gate_parity_and_decrypt(std128, oracle, gate):
    op, ctx, orc, sk, rng = std128["op"], std128["ctx"], std128["orc"], std128["sk"], std128["rng"]
    m1 = np.array([0, 0, 1, 1, 1, 0, 1])
    m2 = np.array([0, 1, 0, 1, 1, 1, 0])
    c1 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m1])
    c2 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m2])
    g = ctx.EvalBinGate(gate, c1, c2)
    assert np.array_equal(g, orc.eval_bin_gate(gate, c1, c2))
    got = [oracle.decrypt(op, sk, r, 4, op.q) for r in g]
    assert got == [TRUTH[gate](int(x), int(y)) for x, y in zip(m1, m2)]


def test_gate_random_inputs_parity(std128):
    op, ctx, orc = std128["op"], std128["ctx"], std128["orc"]
    rs = np.random.default_rng(3)
    c1 = random_cts(rs, 9, op.n, op.q)
    c2 = random_cts(rs, 9, op.n, op.q)
    assert np.array_equal(ctx.EvalBinGate("AND", c1, c2), orc.eval_bin_gate("AND", c1, c2))


def test_gate_errors(std128, capi):
    ctx, op = std128["ctx"], std128["op"]
    c = np.zeros((0, op.n + 1), dtype=np.uint64)
    with pytest.raises(capi.TfheError):
        ctx.EvalBinGate("AND", c, c.copy())


def test_eval_func_parity_all_lut_kinds(std128, oracle):
    """negacyclic (1 bootstrap), periodic and arbitrary (2 bootstraps) LUTs,
    binfhe-base-scheme.cpp:679-789; arbitrary needs q <= N, so q = 512 here."""
    op, ctx, orc, sk, rng = std128["op"], std128["ctx"], std128["orc"], std128["sk"], std128["rng"]
    q = 512
    P = 4
    iv = q // P
    arb = np.array([((i // iv) ** 2 % P) * iv for i in range(q)], dtype=np.uint64)
    half = [(i // iv) * iv + iv // 2 for i in range(q // 2)]
    neg = np.array(half + [q - v for v in half], dtype=np.uint64)
    per = np.array([((i // iv) % 2) * iv for i in range(q)], dtype=np.uint64)
    ms = [0, 1, 2, 3, 1, 2]
    ct = np.stack([oracle.encrypt(op, rng, sk, m, P, q) for m in ms])
    for lut in (arb, neg, per):
        g = ctx.EvalFunc(ct, lut, q=q)
        assert np.array_equal(g, orc.eval_func(ct, lut, q=q))
    luts = np.stack([arb if i % 2 else arb[::-1].copy() for i in range(len(ms))])
    assert np.array_equal(ctx.EvalFunc(ct, luts, q=q), orc.eval_func(ct, luts, q=q))


# ---------------------------------------------------------------- large precision
@pytest.fixture(scope="module")
def sign23(capi, oracle):
    """STD128 logQ=23 throw=1 (time-estimate.cpp:162-163): Q = 2^54 - 77823, 64-bit path."""
    op = oracle.params_from_logq("STD128", False, 23, 0, 0, 1)
    rng = oracle.Rng(9)
    sk, bsk, ksk = oracle.keygen(op, rng)
    cp = capi.params_from_logq("STD128", False, 23, 0, 0, 1)
    ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk)
    yield dict(op=op, cp=cp, sk=sk, ctx=ctx, orc=orc, rng=rng)
    ctx.GPUClean()
    orc.close()


def test_floor_sign_decomp_parity(sign23, oracle):
    op, ctx, orc, sk, rng = sign23["op"], sign23["ctx"], sign23["orc"], sign23["sk"], sign23["rng"]
    Qin = 1 << 17
    p = (op.q // 128 // 2) * (Qin // op.q)
    ms = [0, p // 2 - 8, p // 2 + 8, p - 1]
    ct = np.stack([oracle.encrypt(op, rng, sk, m, p, Qin) for m in ms])
    fl = ctx.EvalFloor(ct, Qin)
    assert np.array_equal(fl, orc.eval_floor(ct, Qin))
    sg = ctx.EvalSign(ct, Qin)
    assert np.array_equal(sg, orc.eval_sign(ct, Qin))
    assert [oracle.decrypt(op, sk, r, 2, op.q) for r in sg] == [int(m >= p // 2) for m in ms]
    d_g, mods_g = ctx.EvalDecomp(ct, Qin)
    d_c, mods_c = orc.eval_decomp(ct, Qin)
    assert mods_g == mods_c
    assert np.array_equal(d_g, d_c)


# ---------------------------------------------------------------- full size property
def test_full_batch_nand_decrypts(std128, oracle):
    """BASELINE config C2 shape (STD128, B=8192): every output decrypts to NAND,
    and a sample equals the oracle bit for bit."""
    op, ctx, orc, sk = std128["op"], std128["ctx"], std128["orc"], std128["sk"]
    rs = np.random.default_rng(4)
    B = 8192
    m1 = rs.integers(0, 2, B)
    m2 = rs.integers(0, 2, B)
    rng = oracle.Rng(123)
    c1 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m1])
    c2 = np.stack([oracle.encrypt(op, rng, sk, int(m), 4, op.q) for m in m2])
    out = ctx.EvalBinGate("NAND", c1, c2)
    dec = np.array([oracle.decrypt(op, sk, r, 4, op.q) for r in out])
    assert np.array_equal(dec, 1 - (m1 & m2))
    idx = [0, 1, 4095, 8191]
    assert np.array_equal(out[idx], orc.eval_bin_gate("NAND", c1[idx], c2[idx]))


def test_key_image_export_import_roundtrip(std128, capi):
    """tfhe_export_key_image -> device buffer -> tfhe_setup_from_key_image (the
    one-process-per-GPU replication path used with RCCL broadcast) yields an
    identical engine."""
    import torch

    ctx, cp = std128["ctx"], std128["cp"]
    nbytes = ctx.info().key_image_bytes
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    ctx.export_key_image(img.data_ptr(), nbytes)
    torch.cuda.synchronize()
    ctx2 = capi.BinFHEContextHIP.from_key_image(cp, img.data_ptr(), nbytes, 0)
    rs = np.random.default_rng(11)
    c1 = random_cts(rs, 6, cp.n, cp.q)
    c2 = random_cts(rs, 6, cp.n, cp.q)
    assert np.array_equal(ctx.EvalBinGate("XOR", c1, c2), ctx2.EvalBinGate("XOR", c1, c2))
    with pytest.raises(capi.TfheError):
        capi.BinFHEContextHIP.from_key_image(cp, img.data_ptr(), nbytes - 1, 0)
    ctx2.GPUClean()


def test_device_gate_entry_matches_host_entry(std128):
    """tfhe_eval_bin_gate_device (bench path, HBM-resident inputs) == host-array entry."""
    import torch

    ctx, cp = std128["ctx"], std128["cp"]
    rs = np.random.default_rng(12)
    c1 = random_cts(rs, 10, cp.n, cp.q)
    c2 = random_cts(rs, 10, cp.n, cp.q)
    d1 = torch.from_numpy(c1.astype(np.int64)).cuda()
    d2 = torch.from_numpy(c2.astype(np.int64)).cuda()
    do = torch.empty_like(d1)
    s = torch.cuda.Stream()
    ctx.EvalBinGateDevice("NAND", 10, d1.data_ptr(), d2.data_ptr(), do.data_ptr(), stream=s.cuda_stream)
    s.synchronize()
    assert np.array_equal(do.cpu().numpy().astype(np.uint64), ctx.EvalBinGate("NAND", c1, c2))


def test_device_then_host_calls_without_sync(std128):
    """Device-resident gates on two user streams, then a host-array gate, with no
    synchronisation between the calls: all three share lane 0's scratch, which the
    engine orders with an event, so every result equals its sequential run."""
    import torch

    ctx, cp = std128["ctx"], std128["cp"]
    rs = np.random.default_rng(13)
    B = 2048
    c1, c2 = random_cts(rs, B, cp.n, cp.q), random_cts(rs, B, cp.n, cp.q)
    h1, h2 = random_cts(rs, 7, cp.n, cp.q), random_cts(rs, 7, cp.n, cp.q)
    want_dev = ctx.EvalBinGate("NAND", c1, c2)
    want_dev2 = ctx.EvalBinGate("AND", c2, c1)
    want_host = ctx.EvalBinGate("OR", h1, h2)
    d1 = torch.from_numpy(c1.astype(np.int64)).cuda()
    d2 = torch.from_numpy(c2.astype(np.int64)).cuda()
    o1, o2 = torch.empty_like(d1), torch.empty_like(d1)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ctx.EvalBinGateDevice("NAND", B, d1.data_ptr(), d2.data_ptr(), o1.data_ptr(), stream=s1.cuda_stream)
    ctx.EvalBinGateDevice("AND", B, d2.data_ptr(), d1.data_ptr(), o2.data_ptr(), stream=s2.cuda_stream)
    got_host = ctx.EvalBinGate("OR", h1, h2)
    s1.synchronize()
    s2.synchronize()
    assert np.array_equal(got_host, want_host)
    assert np.array_equal(o1.cpu().numpy().astype(np.uint64), want_dev)
    assert np.array_equal(o2.cpu().numpy().astype(np.uint64), want_dev2)


# ---------------------------------------------------------------- batch shapes and edge values
@pytest.mark.parametrize("B", [1, 2, 3, 130])
def test_gate_batch_sizes(std128, B):
    """Odd batches leave the fast kernel's last workgroup half idle; B=1 is the scalar API."""
    op, cp, ctx, orc = std128["op"], std128["cp"], std128["ctx"], std128["orc"]
    rs = np.random.default_rng(100 + B)
    c1 = random_cts(rs, B, cp.n, cp.q)
    c2 = random_cts(rs, B, cp.n, cp.q)
    assert np.array_equal(ctx.EvalBinGate("AND", c1, c2), orc.eval_bin_gate("AND", c1, c2))


def test_eval_acc_boundary_values(std128):
    """Accumulator coefficients at the centring boundaries (0, Q>>1, (Q>>1)+-1, Q-1), where a
    wrong canonical/centred representative would change the digit decomposition."""
    op, ctx, orc = std128["op"], std128["ctx"], std128["orc"]
    Q, h = int(op.Q), int(op.Q) >> 1
    edge = np.array([0, 1, h - 1, h, h + 1, Q - 2, Q - 1], dtype=np.uint64)
    rs = np.random.default_rng(3)
    B = 3
    acc = edge[rs.integers(0, len(edge), (B, 2, op.N))]
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    assert np.array_equal(ctx.EvalAcc(a, op.q, acc), orc.eval_acc(a, op.q, acc))


def test_batch_above_chunk_size(std128):
    """A batch larger than the 65536-ciphertext chunk (the reference's max_bootstapping_num)
    spans two device chunks; sampled ciphertexts on both sides equal the oracle."""
    if std128["path"] != "fast":
        pytest.skip("one kernel is enough for the chunking logic")
    op, cp, ctx, orc = std128["op"], std128["cp"], std128["ctx"], std128["orc"]
    rs = np.random.default_rng(9)
    B = 65536 + 5
    c1 = random_cts(rs, B, cp.n, cp.q)
    c2 = random_cts(rs, B, cp.n, cp.q)
    out = ctx.EvalBinGate("OR", c1, c2)
    idx = [0, 1, 65535, 65536, B - 1]
    assert np.array_equal(out[idx], orc.eval_bin_gate("OR", c1[idx], c2[idx]))


@pytest.mark.parametrize("parts", ["1", "2", "3", "7"])
def test_host_pipeline_sub_batches(std128, parts):
    """The host-array runner cuts a shard into sub-batches whose copies (copy stream) overlap
    the kernels (compute stream) through two alternating device I/O sets; every split --
    ragged last sub-batch included -- gives the device-resident result, which equals the
    oracle on a sample.  EvalFunc (one input array, a LUT) and EvalBinGate (two) both."""
    import torch

    if std128["path"] != "fast":
        pytest.skip("one kernel is enough for the pipelining logic")
    op, cp, ctx, orc = std128["op"], std128["cp"], std128["ctx"], std128["orc"]
    rs = np.random.default_rng(17)
    B = 1803
    c1, c2 = random_cts(rs, B, cp.n, cp.q), random_cts(rs, B, cp.n, cp.q)
    d1 = torch.from_numpy(c1.astype(np.int64)).cuda()
    d2 = torch.from_numpy(c2.astype(np.int64)).cuda()
    do = torch.empty_like(d1)
    ctx.EvalBinGateDevice("AND", B, d1.data_ptr(), d2.data_ptr(), do.data_ptr())
    torch.cuda.synchronize()
    want = do.cpu().numpy().astype(np.uint64)
    lut = np.array([(x * 3) % 4 * (cp.q // 4) for x in range(cp.q)], dtype=np.uint64) % cp.q
    with ctx.knobs_set(host_parts=int(parts)):
        got = ctx.EvalBinGate("AND", c1, c2)
        fgot = ctx.EvalFunc(c1, lut)
    assert np.array_equal(got, want)
    idx = [0, 1, B // 2, B - 2, B - 1]
    assert np.array_equal(got[idx], orc.eval_bin_gate("AND", c1[idx], c2[idx]))
    assert np.array_equal(fgot[idx], orc.eval_func(np.ascontiguousarray(c1[idx]), lut))


def test_std128_opt_uses_fast_kernel_exactly(capi, oracle):
    """STD128_OPT (n=502) runs on the specialised kernel too: blind rotation parity with
    random keys (validity is irrelevant for bit-exactness)."""
    op = oracle.params_from_set("STD128_OPT")
    cp = capi.params_from_set("STD128_OPT")
    rs = np.random.default_rng(4)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk)
    B = 3
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    assert np.array_equal(ctx.EvalAcc(a, op.q, acc), orc.eval_acc(a, op.q, acc))
    c1 = random_cts(rs, 4, cp.n, cp.q)
    c2 = random_cts(rs, 4, cp.n, cp.q)
    assert np.array_equal(ctx.EvalBinGate("NOR", c1, c2), orc.eval_bin_gate("NOR", c1, c2))
    ctx.GPUClean()
    orc.close()


def test_key_file_roundtrip(std128, capi, tmp_path):
    """save_key_image -> from_key_file (the on-disk cache of the packed layout) gives an
    identical engine; a wrong parameter set is refused."""
    ctx, cp = std128["ctx"], std128["cp"]
    path = str(tmp_path / "std128.kimg")
    ctx.save_key_image(path)
    ctx2 = capi.BinFHEContextHIP.from_key_file(cp, path)
    rs = np.random.default_rng(21)
    c1 = random_cts(rs, 7, cp.n, cp.q)
    c2 = random_cts(rs, 7, cp.n, cp.q)
    assert np.array_equal(ctx.EvalBinGate("XNOR", c1, c2), ctx2.EvalBinGate("XNOR", c1, c2))
    ctx2.GPUClean()
    with pytest.raises(capi.TfheError, match="parameters differ"):
        capi.BinFHEContextHIP.from_key_file(capi.params_from_set("STD128_OPT"), path)


@pytest.mark.parametrize("pset,path,kernel", [("STD192", "f64", 3), ("STD192", "f64-nofold", 0), ("STD192", "generic", 0),
                                              ("STD192Q_OPT", "f64", 3), ("STD128Q", "f64", 3),
                                              ("STD128Q", "f64-one-workgroup", 3), ("STD128Q", "f64-exactonly", 0),
                                              ("STD128Q", "generic-v2", 0), ("STD192", "generic-v1", 0)])
def test_n2048_blind_rotation_parity(capi, oracle, pset, path, kernel):
    """STD192 (Q = 2^37 - 2^17 + 1) and STD128Q (Q = 2^50 - 2^14 + 1, the reducing variant),
    N = 2048, run on the exact-FP64 kernel by default with the top digit's transforms eliminated
    (STD128Q at this batch: the two-workgroup f64wduo; duo = 0 keeps f64w) and on the u64 generic
    kernel with TFHE_FORCE_GENERIC=1; all equal the oracle, including accumulator boundary values.
    STD128Q's top digit is not always exact (centred c in [2^49 - 2^24, Q/2) leaves a residual), so
    its fold runs the WRAP correction: Q/2 - 1 and Q/2 - 5000 put such coefficients in round 0, so the
    correction runs.  Unfolded contexts (TFHE_F64_FOLD=0, or =1 on STD128Q: exact sets only) run the
    generic kernel since round 5 retired the slot-layout FP64 kernel."""
    op = oracle.params_from_set(pset)
    cp = capi.params_from_set(pset)
    rs = np.random.default_rng(5)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    env = {"generic": ("TFHE_FORCE_GENERIC", "1"), "f64-nofold": ("TFHE_F64_FOLD", "0"),
           "f64-exactonly": ("TFHE_F64_FOLD", "1"),
           "generic-v2": ("TFHE_FORCE_GENERIC", "1"), "generic-v1": ("TFHE_FORCE_GENERIC", "1")}.get(path)
    knob = {"generic-v2": {"generic": 2}, "generic-v1": {"generic": 1}, "f64-one-workgroup": {"duo": 0}}.get(path, {})
    if env:
        os.environ[env[0]] = env[1]
    try:  # the environment is read at setup (tfhe_knobs); the generic kernel's form is a knob
        ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk, memo=("n2048", pset))
        assert ctx.info().br_kernel == kernel
        ctx.set_knobs(**knob)
        B = 2
        a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
        acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
        acc[1, :, :6] = [0, op.Q - 1, op.Q >> 1, (op.Q >> 1) + 1, (op.Q >> 1) - 1, (op.Q >> 1) - 5000]
        assert np.array_equal(ctx.EvalAcc(a, op.q, acc), orc.eval_acc(a, op.q, acc))
    finally:
        if env:
            os.environ.pop(env[0], None)
    ctx.GPUClean()
    orc.close()



@pytest.mark.parametrize("arb,logq,path,kernel", [(True, 12, "sf", 5), (False, 23, "sf", 5), (True, 12, "gen3sf", 5),
                                                   (False, 23, "gen3sf", 5), (True, 12, "generic", 0),
                                                   (False, 23, "generic", 0)])
def test_logq_blind_rotation_parity(capi, oracle, arb, logq, path, kernel):
    """The logQ contexts (Q = 2^54 - 77823, N = 2048, throw = 1: C3 logQ=12 with one 27-bit digit
    per polynomial, C5b logQ=23 with two 18-bit digits) run on the special-form u64 kernel by
    default (constants as (w, w 2^31 mod Q), five multiplies per product) and on the Shoup gen3
    kernel with TFHE_SF=0; all equal the oracle, for accumulator and key boundary values (0, Q-1, the
    centring threshold, the largest top digits) and several a-moduli."""
    op = oracle.params_from_logq("STD128", arb, logq, 0, 0, 1)
    cp = capi.params_from_logq("STD128", arb, logq, 0, 0, 1)
    rs = np.random.default_rng(logq)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    bsk[: 4 * op.N] = np.array([0, op.Q - 1, op.Q >> 1, (op.Q >> 1) + 1], dtype=np.uint64).repeat(op.N)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    env = {"generic": ("TFHE_SF", "0"), "gen3sf": ("TFHE_SF2", "0")}.get(path)
    if env:
        os.environ[env[0]] = env[1]
    try:  # both read at setup (TFHE_SF2 into the sf2 knob)
        ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk, memo=("logq", arb, logq))
        assert ctx.info().br_kernel == kernel
        B = 3
        acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
        half = op.Q >> 1
        acc[0, :, :8] = [0, op.Q - 1, half, half + 1, half - 1, 1, op.Q - 2, half + 2]
        acc[1] = np.where(rs.integers(0, 2, (2, op.N)) == 1, half, half + 1).astype(np.uint64)  # extreme digits
        for amod in (op.q, 2 * op.N):
            a = rs.integers(0, amod, (B, op.n), dtype=np.uint64)
            assert np.array_equal(ctx.EvalAcc(a, amod, acc), orc.eval_acc(a, amod, acc))
    finally:
        if env:
            os.environ.pop(env[0], None)
    ctx.GPUClean()
    orc.close()


@pytest.mark.parametrize("shape,path", [(s, p) for s in ("logq11", "logq11-thr1", "arb11-thr1", "STD128_AP")
                                        for p in ("fast", "generic")])
def test_n1024_digit_shapes_parity(capi, oracle, shape, path):
    """The four-wavefront kernel's other digit shapes (N = 1024, Q = 2^27 - 2^11 + 1):
    logQ = 11 without a thrown digit (six 5-bit digits, top digit eliminated), logQ = 11 with
    one thrown digit (five transformed digits, the thrown one's carry kept; EvalFloor's context
    in the reference's time-estimate.cpp:100) and STD128_AP (three 9-bit digits whose top
    digit wraps, so none is eliminated).  Fast kernel (br_kernel 1) and generic v2
    (TFHE_FORCE_GENERIC=1) equal the oracle for accumulator boundary values and both a-moduli."""
    if shape == "STD128_AP":
        op, cp = oracle.params_from_set(shape), capi.params_from_set(shape)
    else:
        arb, thr = shape.startswith("arb"), 1 if shape.endswith("thr1") else 0
        op = oracle.params_from_logq("STD128", arb, 11, 0, 0, thr)
        cp = capi.params_from_logq("STD128", arb, 11, 0, 0, thr)
    rs = np.random.default_rng(17)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    bsk[: 4 * op.N] = np.array([0, op.Q - 1, op.Q >> 1, (op.Q >> 1) + 1], dtype=np.uint64).repeat(op.N)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    if path == "generic":
        os.environ["TFHE_FORCE_GENERIC"] = "1"
    try:
        ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk, memo=("n1024", shape))
    finally:
        os.environ.pop("TFHE_FORCE_GENERIC", None)
    assert ctx.info().br_kernel == (1 if path == "fast" else 0)
    B = 3
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    half = op.Q >> 1
    acc[0, :, :8] = [0, op.Q - 1, half, half + 1, half - 1, 1, op.Q - 2, half + 2]
    acc[1] = np.where(rs.integers(0, 2, (2, op.N)) == 1, half, half + 1).astype(np.uint64)  # extreme digits
    for amod in (op.q, 2 * op.N):
        a = rs.integers(0, amod, (B, op.n), dtype=np.uint64)
        assert np.array_equal(ctx.EvalAcc(a, amod, acc), orc.eval_acc(a, amod, acc))
    if shape == "logq11-thr1":  # EvalFloor end to end (the reference example's call)
        ct = random_cts(rs, 4, cp.n, cp.q)
        assert np.array_equal(ctx.EvalFloor(ct, cp.q, 1), orc.eval_floor(ct, cp.q, 1))
    ctx.GPUClean()
    orc.close()


@pytest.mark.parametrize("pset", ["STD128Q", "STD128Q_OPT"])
def test_wrap_correction_late_round(capi, oracle, pset):
    """The STD128Q fold's WRAP correction in the LAST round (vote flag of round parity
    (n-1) & 1, after n-1 rounds of flag resets): a_i = 0 for i < n-1 makes those rounds add
    (X^0 - 1)(...) = 0, so the accumulator keeps its boundary values (centred c just below Q/2,
    where the reference's signed digits leave a residual) until the last round, whose
    a_{n-1} is random.  Equal to the oracle."""
    op = oracle.params_from_set(pset)
    cp = capi.params_from_set(pset)
    rs = np.random.default_rng(11)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk)
    assert ctx.info().br_kernel == 3
    B = 3
    a = np.zeros((B, op.n), dtype=np.uint64)
    a[:, -1] = rs.integers(1, op.q, B, dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    half = op.Q >> 1
    acc[:, :, 10:20] = (half - 1 - rs.integers(0, 1 << 23, (B, 2, 10))).astype(np.uint64)
    acc[2] = rs.integers(0, op.Q, (2, op.N), dtype=np.uint64)  # a ciphertext without residuals
    assert np.array_equal(ctx.EvalAcc(a, op.q, acc), orc.eval_acc(a, op.q, acc))
    ctx.GPUClean()
    orc.close()

@pytest.mark.parametrize("pset", ["STD128Q_OPT", "STD192", "STD128", "LOGQ54"])
def test_repeated_calls_stable(capi, oracle, pset):
    """The same EvalAcc six times on one context, every result equal to the oracle: f64w (STD128Q,
    STD192) once went wrong in some calls only -- a missing barrier between its prologue transform
    and round 0 (profiles/r03e/summary.txt, tests/test_gpu_f64w_race.py) -- and one call per test
    did not show it reliably.  STD128 (fast4) and the 54-bit-Q logQ context (sf2) run the same
    check."""
    if pset == "LOGQ54":
        op = oracle.params_from_logq("STD128", False, 23, 0, 0, 1)
        cp = capi.params_from_logq("STD128", False, 23, 0, 0, 1)
    else:
        op = oracle.params_from_set(pset)
        cp = capi.params_from_set(pset)
    rs = np.random.default_rng(12)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk)
    B = 3
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    acc[:2, :, 10:20] = ((op.Q >> 1) - 1 - rs.integers(0, 1 << 23, (2, 2, 10))).astype(np.uint64)
    want = orc.eval_acc(a, op.q, acc)
    bad = [r for r in range(6) if not np.array_equal(ctx.EvalAcc(a, op.q, acc), want)]
    assert bad == [], f"calls {bad} differ from the oracle"
    ctx.GPUClean()
    orc.close()


def _prime_1_mod(m, bits):
    """Largest prime p < 2^bits with p = 1 (mod m) (deterministic Miller-Rabin for 64-bit)."""
    def is_prime(n):
        if n < 2:
            return False
        d, s = n - 1, 0
        while d % 2 == 0:
            d //= 2
            s += 1
        for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
            x = pow(a, d, n)
            if x in (1, n - 1) or a % n == 0:
                continue
            for _ in range(s - 1):
                x = x * x % n
                if x == n - 1:
                    break
            else:
                return False
        return True
    p = ((1 << bits) - 1) // m * m + 1
    while not is_prime(p):
        p -= m
    return p


@pytest.mark.parametrize("bits,baseG_log", [(35, 12), (45, 15)])
def test_custom_modulus_n1024_f64_parity(capi, oracle, bits, baseG_log):
    """User-defined parameters (C-ABI tfhe_params_finish) with a 35-bit / 45-bit Q at N=1024
    exercise the exact-FP64 kernel's N=1024 instances (plain and reducing)."""
    import ctypes as C

    from tfhe_amd import capi as raw

    cp = capi.params_from_set("STD128")
    cp.Q = _prime_1_mod(2 * cp.N, bits)
    cp.baseG = 1 << baseG_log
    cp.digitsG = cp.dG2 = 0
    raw.check(raw.lib().tfhe_params_finish(C.byref(cp)), "tfhe_params_finish")
    op = oracle.params_from_set("STD128")
    for k in ("Q", "baseG", "digitsG", "dG2", "numDigitsToThrow"):
        setattr(op, k, getattr(cp, k))
    op.logG = baseG_log
    rs = np.random.default_rng(bits)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk)
    B = 3
    a = rs.integers(0, op.q, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    assert np.array_equal(ctx.EvalAcc(a, op.q, acc), orc.eval_acc(a, op.q, acc))
    ctx.GPUClean()
    orc.close()


def test_host_array_unreduced_inputs_take_the_wide_wire(capi, oracle):
    """The host-array runner sends arrays in u16 / u32 words when their modulus allows (engine.hip
    h2d_staged); an unreduced input (a >= a_mod, acc >= Q -- the kernels reduce both) must fall
    back to u64 and give the same result as the reduced one."""
    op = oracle.params_from_set("STD128")
    cp = capi.params_from_set("STD128")
    rs = np.random.default_rng(41)
    bsk = rs.integers(0, op.Q, cp.bsk_words(), dtype=np.uint64)
    ksk = rs.integers(0, op.qKS, cp.ksk_words(), dtype=np.uint64)
    ctx, orc = make_pair(capi, oracle, op, cp, bsk, ksk)
    B, amod = 6, op.q
    a = rs.integers(0, amod, (B, op.n), dtype=np.uint64)
    acc = rs.integers(0, op.Q, (B, 2, op.N), dtype=np.uint64)
    want = orc.eval_acc(a, amod, acc)
    assert np.array_equal(ctx.EvalAcc(a, amod, acc), want)
    a_big = a + np.uint64(amod) * rs.integers(1, 1 << 40, (B, op.n), dtype=np.uint64)
    acc_big = acc + np.uint64(op.Q) * rs.integers(0, 1 << 30, (B, 2, op.N), dtype=np.uint64)
    assert np.array_equal(ctx.EvalAcc(a_big, amod, acc_big), want)
    ext = rs.integers(0, op.Q, (B, op.N + 1), dtype=np.uint64)
    assert np.array_equal(ctx.MKMSwitch(ext, op.q), orc.mkm_switch(ext, op.q))
    ctx.GPUClean()
    orc.close()
