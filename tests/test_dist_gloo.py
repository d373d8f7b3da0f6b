"""World-size-2 torch.distributed (gloo, CPU) tests of the multi-rank path:
contiguous sharding, the key-image broadcast, max-over-ranks timing, and an
end-to-end sharded batch (each rank bootstraps its shard with the CPU oracle,
standing in for its GPU) that must equal the unsharded result.  The split itself is
the engine's own code: tfhe_shard_range across ranks, and inside each rank the
host-thread runner of a multi-device context (tfhe_host_shard_selftest: the same
run_shards the device calls use, with no GPU work), including its error path."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tfhe_amd import dist as tdist
    import pyoracle

    dev = torch.device("cpu")
    # 1) key image broadcast (stand-in bytes of a real image size)
    nbytes = 4096 + 17
    img = None
    if rank == 0:
        g = torch.Generator().manual_seed(7)
        img = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g)
    got = tdist.broadcast_key_image(img, nbytes if rank == 0 else None, dev)
    torch.save(got, os.path.join(outdir, f"img{rank}.pt"))
    # 2) max over ranks
    m = tdist.max_over_ranks(1.5 + rank, dev)
    # 3) sharded batch: TOY keys from a shared seed, NAND over B=5 pairs
    p = pyoracle.params_from_set("TOY")
    rng = pyoracle.Rng(99)
    sk, bsk, ksk = pyoracle.keygen(p, rng)
    B = 5
    c1 = np.stack([pyoracle.encrypt(p, rng, sk, i % 2, 4, p.q) for i in range(B)])
    c2 = np.stack([pyoracle.encrypt(p, rng, sk, (i // 2) % 2, 4, p.q) for i in range(B)])
    lo, hi = tdist.shard_range(B, world, rank)
    # the engine's in-process split of this rank's shard over 2 devices (global spans)
    BIG = 8191
    blo, bhi = tdist.shard_range(BIG, world, rank)
    dev_spans = [(blo + l, n) for l, n in tdist.device_shards(bhi - blo, 2)]
    all_dev = [None] * world
    dist.all_gather_object(all_dev, dev_spans)
    orc = pyoracle.Oracle(p, bsk, ksk, threads=1)
    part = orc.eval_bin_gate("NAND", c1[lo:hi], c2[lo:hi]) if hi > lo else np.zeros((0, p.n + 1), np.uint64)
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, part))
    total = tdist.sum_over_ranks(hi - lo, dev)
    if rank == 0:
        full = np.concatenate([x[2] for x in sorted(parts, key=lambda t: t[0])])
        ref = orc.eval_bin_gate("NAND", c1, c2)
        np.save(os.path.join(outdir, "sharded.npy"), full)
        np.save(os.path.join(outdir, "ref.npy"), ref)
        with open(os.path.join(outdir, "meta.txt"), "w") as f:
            f.write(f"{m} {total}\n")
        spans = sorted(x for r in all_dev for x in r)
        with open(os.path.join(outdir, "dev_spans.txt"), "w") as f:
            f.write(" ".join(f"{l}:{n}" for l, n in spans) + f" total={BIG}\n")
    orc.close()
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_exactly():
    sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))
    from tfhe_amd.dist import shard_range

    for total in (0, 1, 7, 8192, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for a, b in zip(spans, spans[1:]):
                assert a[1] == b[0]
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def test_gloo_world2_broadcast_and_sharded_batch(tmp_path, oracle):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    a = torch.load(tmp_path / "img0.pt")
    b = torch.load(tmp_path / "img1.pt")
    assert torch.equal(a, b) and a.numel() == 4096 + 17
    m, total = open(tmp_path / "meta.txt").read().split()
    assert float(m) == 2.5 and int(total) == 5
    assert np.array_equal(np.load(tmp_path / "sharded.npy"), np.load(tmp_path / "ref.npy"))
    # 4 device spans (2 ranks x 2 devices) partition the batch in order, sizes within 1
    *parts, tot = open(tmp_path / "dev_spans.txt").read().split()
    spans = [tuple(map(int, x.split(":"))) for x in parts]
    assert int(tot.split("=")[1]) == sum(n for _, n in spans) == 8191
    assert spans[0][0] == 0 and all(l + n == l2 for (l, n), (l2, _) in zip(spans, spans[1:]))
    assert max(n for _, n in spans) - min(n for _, n in spans) <= 1


def test_engine_device_split_and_error_propagation():
    """The multi-device runner of a tfhe_setup(num_gpus) context (run_shards, one host thread
    per device): contiguous balanced spans, a batch below 2 per device stays on device 0, and a
    failing device's error comes back with its shard."""
    sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))
    from tfhe_amd.capi import TfheError
    from tfhe_amd.dist import device_shards

    for total in (0, 1, 5, 16, 8192, 65537):
        for devices in (1, 2, 3, 8):
            spans = device_shards(total, devices)
            if devices == 1 or total < 2 * devices:
                assert spans[0] == (0, total) and all(n == 0 for _, n in spans[1:])
                continue
            assert spans[0][0] == 0 and sum(n for _, n in spans) == total
            assert all(l + n == l2 for (l, n), (l2, _) in zip(spans, spans[1:]))
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1
    with pytest.raises(TfheError, match=r"device 1: injected fault on shard \[10, 20\)"):
        device_shards(30, 3, fail_device=1)
    with pytest.raises(TfheError, match=r"device 7: injected fault on shard \[7168, 8192\)"):
        device_shards(8192, 8, fail_device=7)
    assert device_shards(30, 3, fail_device=5)[2] == (20, 10)  # no such device: no failure


def _bench_check_worker(rank, world, port, outdir, corrupt_rank):
    """bench.py's per-rank output check: each rank's first outputs (the oracle stands in for its
    GPU; rank `corrupt_rank` flips one bit) are gathered and rank 0 checks them all."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tfhe-gpu_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import pyoracle

    cfg = {"ctx": ("set", "TOY"), "op": "gate"}
    p = pyoracle.params_from_set("TOY")
    rng = pyoracle.Rng(5)
    sk, bsk, ksk = pyoracle.keygen(p, rng)
    rs = np.random.default_rng(100 + rank)
    c1 = rs.integers(0, p.q, (3, p.n + 1), dtype=np.uint64)
    c2 = rs.integers(0, p.q, (3, p.n + 1), dtype=np.uint64)
    orc = pyoracle.Oracle(p, bsk, ksk, threads=1)
    out = orc.eval_bin_gate("NAND", c1, c2)
    orc.close()
    if rank == corrupt_rank:
        out[1, 3] ^= np.uint64(1)
    per_rank = bench.gather_rank_samples([c1, c2, out], world, torch.device("cpu"))
    if rank == 0:
        rec = bench.oracle_sample_check(cfg, bsk, ksk, per_rank, threads=1)
        ok, failed = bench.parity_verdict(None, None, None, rec)
        with open(os.path.join(outdir, "check.txt"), "w") as f:
            f.write(f"{rec['ranks_checked']} {rec['ranks_passed']} {int(ok)} {','.join(failed)}\n")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("corrupt_rank", [-1, 1])
def test_gloo_world2_bench_rank_sample_check(tmp_path, oracle, corrupt_rank):
    mp.spawn(_bench_check_worker, args=(2, _free_port(), str(tmp_path), corrupt_rank), nprocs=2, join=True)
    checked, passed, ok, *failed = open(tmp_path / "check.txt").read().split()
    assert int(checked) == 2
    if corrupt_rank < 0:
        assert int(passed) == 2 and ok == "1" and not failed
    else:
        assert int(passed) == 1 and ok == "0" and failed == ["oracle_sample"]
