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
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        return local
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    width = max(b - a for a, b in sizes)
    if width * world == n_total:  # even shards (e.g. C3: 256 = 8 x 32): gather in place, no pad/trim
        out = torch.empty((n_total,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    pad = torch.zeros((width,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    pad[: local.shape[0]] = local
    out = torch.empty((world * width,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r * width: r * width + (b - a)] for r, (a, b) in enumerate(sizes)], 0)


def sharded_step(predict, x_local: torch.Tensor, T: torch.Tensor, n_total: int, group=None,
                 gather_maps: bool = False):
    """One data-parallel step of the path: this rank's shard of the global batch
    (shard_range order) through `predict(x, T) -> (maps [b, ...], scores [b])`, then
    the path's only exchange, the all-gather of the per-image scores (and of the
    maps when the caller needs them, e.g. for metrics_eval on rank 0).
    Returns (local maps, local scores, global scores [n_total], global maps or None)."""
    maps, scores = predict(x_local, T)
    s_all = gather_rows(scores, n_total, group)
    m_all = gather_rows(maps, n_total, group) if gather_maps else None
    return maps, scores, s_all, m_all


def verify_gather(predict, images_of, s_all: torch.Tensor, s_local: torch.Tensor, n_total: int, group=None,
                  checker: int = 0) -> dict:
    """Self-check of a data-parallel step after the fact, so an N-rank run proves its
    own gathered result: (1) every rank finds its local scores, bit for bit, at its
    shard_range slice of the gathered vector; (2) rank `checker` recomputes the shard of
    the last other rank with images (a foreign shard it never predicted in the step) with
    `predict(images_of(a, b))` and compares it bit for bit with that slice. Per-image
    results do not depend on batch composition (tests/test_e2e_gpu.py), so the foreign
    shard's bits are the same whoever computes them. Both flags are MIN-reduced over
    the ranks, so every rank returns the same verdict:
    {"backend", "world", "own_slice_verified", "gather_verified", "checked_shard"}."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = shard_range(n_total, rank, world)
    own = bool(torch.equal(s_all[a:b], s_local))
    foreign = True
    # the last rank other than the checker with a non-empty shard (the checker's own if none)
    cand = [r for r in range(world) if r != checker and shard_range(n_total, r, world)[1] > shard_range(n_total, r, world)[0]]
    who = cand[-1] if cand else checker
    fa, fb = shard_range(n_total, who, world)
    if rank == checker and fb > fa:
        ref = predict(images_of(fa, fb))
        foreign = bool(torch.equal(s_all[fa:fb], ref.to(s_all.device)))
    flags = torch.tensor([int(own), int(foreign)], dtype=torch.int32, device=s_all.device)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN, group=group)
    return {"backend": str(dist.get_backend(group)), "world": world, "own_slice_verified": bool(flags[0]),
            "gather_verified": bool(flags[1]), "checked_shard": {"rank": who, "images": [fa, fb],
                                                                 "checked_by": checker}}


def gather_rows_to(local: torch.Tensor, n_total: int, dst: int = 0, group=None, host_staging=None):
    """Gather variable-size row shards (shard_range order) onto rank `dst` only: returns
    the global [n_total, ...] tensor there and None on the other ranks. For results only
    one rank consumes (the harness's pixel maps before metrics_eval): 1/world of
    gather_rows' receive traffic. An empty local shard (n_total < world) still takes
    part, with zero rows of the right shape.
    host_staging: None = by backend (gloo's gather takes host tensors only -- the one-GPU
    rehearsal of the multi-rank harness, every rank on cuda:0 over gloo; RCCL gathers
    device memory directly); False = gather `local` where it lives (the RCCL branch; the
    CPU tests force it with host tensors over gloo), True = stage through host memory."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        return local
    rank = dist.get_rank(group)
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    width = max(b - a for a, b in sizes)
    host = str(dist.get_backend(group)) == "gloo" if host_staging is None else bool(host_staging)
    pad = torch.zeros((width,) + tuple(local.shape[1:]), device="cpu" if host else local.device, dtype=local.dtype)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([bufs[r][: b - a] for r, (a, b) in enumerate(sizes)], 0).to(local.device)
