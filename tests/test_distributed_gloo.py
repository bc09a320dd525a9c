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


class _StandIn:
    """CPU stand-in for AdaptedCLIP.predict: per-image map and score that depend only
    on that image (the property the image sharding relies on)."""

    def predict(self, image, T, domain="Industrial", streams=1):
        maps = image.mean(1) * T.sum()
        return maps, maps.mean((1, 2)) + image[:, 0, 0, 0]


def _sharded_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aa-clip_amd"))
    import test as harness
    from aaclip.parallel import sharded_step
    from dataset import get_dataset
    model = _StandIn()
    T = torch.full((4, 2), 0.5)
    # bench step: this rank's shard_range slice of one global batch -> gathered scores
    g = torch.Generator().manual_seed(111)
    x_global = torch.randn(n, 3, 28, 28, generator=g)
    a, b = shard_range(n, rank, world)
    _, s_loc, s_all, m_all = sharded_step(model.predict, x_global[a:b], T, n, gather_maps=True)
    # the bench's N-rank self-check: own slices + the last rank's shard recomputed on rank 0
    from aaclip.parallel import verify_gather
    pred = lambda xi: model.predict(xi, T)[1]  # noqa: E731
    check = verify_gather(pred, lambda i0, i1: x_global[i0:i1], s_all, s_loc, n)
    bad = s_all.clone()
    fa, fb = check["checked_shard"]["images"]
    bad[fb - 1] += 1.0  # a corrupted gather (last image of the checked shard) must be caught
    check_bad = verify_gather(pred, lambda i0, i1: x_global[i0:i1], bad, s_loc, n)
    # harness: one class's dataset sharded by image, gathered before metrics
    ds = get_dataset("synthetic", 28, None, -1, "test", synthetic_n=n)["bottle"]
    sub = torch.utils.data.Subset(ds, range(*shard_range(n, rank, world)))
    loader = torch.utils.data.DataLoader(sub, batch_size=3, shuffle=False)
    masks, labels, preds, preds_image, names = harness.get_predictions(model, T, loader, torch.device("cpu"), 28,
                                                                       dataset="synthetic", n_total=n)
    if rank == 0:  # the class is gathered onto rank 0 (which runs metrics_eval)
        q.put((rank, s_all.tolist(), m_all.sum().item(), masks.sum().item(), labels.tolist(), preds.sum().item(),
               preds_image.tolist(), names, check, check_bad))
    else:
        assert masks is None and labels is None and preds is None and preds_image is None and names is None
        q.put((rank, s_all.tolist(), m_all.sum().item(), None, None, None, None, None, check, check_bad))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [8, 7, 1])
def test_gloo_world2_sharded_step_and_harness(n):
    """The bench's data-parallel step (aaclip.parallel.sharded_step) and the harness's
    sharded get_predictions on 2 gloo ranks with a CPU stand-in predictor: every rank
    ends with the unsharded run's gathered scores and maps (the bench step), rank 0 with
    exactly the unsharded run's class masks, labels, maps, scores and file names (the
    harness gathers onto rank 0 only), including a rank with an EMPTY shard."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aa-clip_amd"))
    import test as harness
    from dataset import get_dataset
    model = _StandIn()
    T = torch.full((4, 2), 0.5)
    g = torch.Generator().manual_seed(111)
    x_global = torch.randn(n, 3, 28, 28, generator=g)
    ref_maps, ref_scores = model.predict(x_global, T)
    ds = get_dataset("synthetic", 28, None, -1, "test", synthetic_n=n)["bottle"]
    ref = harness.get_predictions(model, T, torch.utils.data.DataLoader(ds, batch_size=3, shuffle=False),
                                  torch.device("cpu"), 28, dataset="synthetic")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, s_all, m_sum, mk_sum, labels, p_sum, pi, names, check, check_bad in out:
        assert check["backend"] == "gloo" and check["world"] == 2
        assert check["gather_verified"] and check["own_slice_verified"], check
        # the corruption sits in the checked shard and in its owner's own slice
        assert not check_bad["gather_verified"] and not check_bad["own_slice_verified"], check_bad
        assert s_all == ref_scores.tolist()
        assert m_sum == ref_maps.sum().item()
        if mk_sum is None:
            continue
        assert mk_sum == ref[0].sum().item() and labels == ref[1].tolist()
        assert p_sum == ref[2].sum().item() and pi == ref[3].tolist() and names == ref[4]


def _gather_to_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from aaclip.parallel import gather_rows_to
    a, b = shard_range(n, rank, world)
    local = torch.arange(a, b, dtype=torch.float32)[:, None, None].expand(-1, 3, 5).contiguous() * 0.25
    res = {}
    for staging in (False, True, None):  # False: the device-tensor (RCCL) branch, no host copy
        out = gather_rows_to(local, n, dst=1, host_staging=staging)
        res[str(staging)] = None if out is None else (list(out.shape), out[:, 0, 0].tolist(), str(out.device))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [7, 8, 1])
def test_gloo_world2_gather_rows_to_both_branches(n):
    """gather_rows_to onto rank 1 through BOTH of its branches: the direct gather of the
    tensor where it lives (the branch RCCL takes on the MI355X node; forced here with host
    tensors over gloo) and the host-staged one (gloo rehearsals on cuda:0). Uneven (4 + 3),
    even and one-empty-shard cases; only dst receives."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_to_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v is None for v in out[0].values())
    for v in out[1].values():
        assert v == ([n, 3, 5], [i * 0.25 for i in range(n)], "cpu")
