"""Image-sharded data parallelism for the anomaly-map path.

Images are independent units: each rank (one process per GPU, torchrun-style)
owns a contiguous, balanced shard of the global batch, runs the whole path on
it with replicated weights, and the only exchange is an all-gather of the
per-image results (image scores; optionally pixel maps) — RCCL over xGMI on the
MI355X node ("nccl" backend), gloo for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced shard [start, stop) of n items for `rank` of `world`."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather variable-size row shards (produced by shard_range order) into the
    global [n_total, ...] tensor on every rank. One collective: shards are padded
    to the largest shard, gathered with all_gather_into_tensor, then trimmed."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    width = max(b - a for a, b in sizes)
    pad = torch.zeros((width,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    pad[: local.shape[0]] = local
    out = torch.empty((world * width,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r * width: r * width + (b - a)] for r, (a, b) in enumerate(sizes)], 0)
