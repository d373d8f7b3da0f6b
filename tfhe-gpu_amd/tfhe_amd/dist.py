"""Multi-GPU helpers: one process per GPU over torch.distributed.

The bootstrap path shards with no exchange step (independent ciphertexts,
SURVEY.md 8(e)), so the only collectives are at setup and for timing:

* ``broadcast_key_image``: rank 0's packed device key image (NTT-domain BSK,
  packed KSK, tables; ``tfhe_export_key_image``) is broadcast once.  With the
  "nccl" backend (RCCL on ROCm) this moves device memory over xGMI; the reference
  instead replicates keys host-to-device per GPU (bootstrapping.cu:1005-1069).
* ``shard_range``: contiguous shards [g*B/G, (g+1)*B/G) (the reference deals
  SM_count-sized chunks round-robin, bootstrapping.cu:1617).
* ``device_shards``: the engine's in-process split over the devices of one
  tfhe_setup(num_gpus) context (one host thread per device).
* ``max_over_ranks``: the bench's whole-job time is the slowest rank's.

Everything here is backend-agnostic and is exercised on CPU with gloo
(tests/test_dist_gloo.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of `total` units for `rank` of `world` (sizes differ by <= 1): the engine's
    own split (tfhe_shard_range, the one tfhe_setup(num_gpus) contexts use across devices)."""
    import ctypes as C

    from .capi import lib

    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    lo, hi = C.c_size_t(), C.c_size_t()
    if lib().tfhe_shard_range(total, world, rank, C.byref(lo), C.byref(hi)) != 0:
        raise ValueError("bad world/rank")
    return lo.value, hi.value


def device_shards(total: int, devices: int, fail_device: int = -1) -> list[tuple[int, int]]:
    """(lo, count) per device of the engine's in-process split of `total` ciphertexts over
    `devices` devices -- the host-thread runner a tfhe_setup(num_gpus) context uses
    (tfhe_host_shard_selftest runs it with no GPU work).  fail_device >= 0 injects a failure on
    that device's shard; the engine's error is raised as TfheError."""
    import ctypes as C

    from .capi import check, lib

    spans = (C.c_size_t * (2 * devices))()
    check(lib().tfhe_host_shard_selftest(total, devices, fail_device, spans), "tfhe_host_shard_selftest")
    return [(spans[2 * g], spans[2 * g + 1]) for g in range(devices)]


def broadcast_key_image(image: torch.Tensor | None, nbytes: int | None, device, src: int = 0) -> torch.Tensor:
    """Broadcast a uint8 key image from `src`.  On src pass the filled tensor; elsewhere
    pass None (its size is broadcast first).  Returns the tensor holding the image."""
    rank = dist.get_rank()
    size = torch.tensor([nbytes if rank == src else 0], dtype=torch.int64, device=device)
    dist.broadcast(size, src)
    n = int(size.item())
    if rank != src:
        image = torch.empty(n, dtype=torch.uint8, device=device)
    elif image is None or image.numel() != n or image.dtype != torch.uint8:
        raise ValueError("source rank must pass a uint8 image of nbytes")
    dist.broadcast(image, src)
    return image


def max_over_ranks(x: float, device) -> float:
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(x: float, device) -> list[float]:
    """Every rank's value of x, in rank order (per-rank kernel times in the bench line)."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def sum_over_ranks(x: int, device) -> int:
    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
