"""N>1 path on the CPU: world_size-2 gloo ranks shard the image batch with
shard_range and reassemble per-image results with gather_rows (the RCCL
all-gather of the MI355X run, same code path, gloo backend)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aaclip.parallel import gather_rows, shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 32, 256, 257):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = shard_range(n, rank, world)
    # each rank "scores" its own images (image index -> score), like the per-rank predict()
    local_scores = torch.arange(a, b, dtype=torch.float32) * 0.5 + 1.0
    local_maps = torch.arange(a, b, dtype=torch.float32)[:, None, None].expand(-1, 4, 4).contiguous()
    s = gather_rows(local_scores, n)
    m = gather_rows(local_maps, n)
    q.put((rank, s.tolist(), m[:, 0, 0].tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [32, 33])
def test_gloo_world2_gather(n):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, s, m in out:
        assert s == [i * 0.5 + 1.0 for i in range(n)]
        assert m == [float(i) for i in range(n)]
