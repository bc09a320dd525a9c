"""The RCCL ("nccl" backend) code path on the MI355X, at the world size a one-GPU box
allows (1 rank): process-group init bound to the device exactly as bench.py and the
harness do it (`init_process_group("nccl", device_id=...)`), then the collectives the
sharded path issues -- all_gather_into_tensor (parallel.gather_rows), gather
(parallel.gather_rows_to) and the MIN all_reduce of parallel.verify_gather -- on device
tensors, and verify_gather over a real VisualEngine predict. RCCL refuses two ranks on
one device, so N > 1 over RCCL is the driver's 8-GPU run; the N-rank logic itself is
covered by tests/test_distributed_gloo.py."""
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_group(dev):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 2000))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    yield dist.group.WORLD
    dist.destroy_process_group()


def test_rccl_collectives(dev, rccl_group):
    assert dist.get_backend() == "nccl"
    x = torch.arange(96, device=dev, dtype=torch.float32).view(12, 8)
    out = torch.empty_like(x)
    dist.all_gather_into_tensor(out, x)
    torch.cuda.synchronize()
    assert torch.equal(out, x)
    bufs = [torch.empty_like(x)]
    dist.gather(x, gather_list=bufs, dst=0)
    assert torch.equal(bufs[0], x)
    flags = torch.tensor([1, 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    assert flags.tolist() == [1, 0]


def test_rccl_verify_gather_real_predict(dev, rccl_group):
    """parallel.sharded_step + verify_gather on the HIP engine over RCCL: the line
    bench.py emits as `distributed` (world 1: the own slice and the recomputed shard
    are the same images, so this checks the plumbing and the bit-reproducibility)."""
    from aaclip.engine import VisualEngine
    from aaclip.parallel import sharded_step, verify_gather
    from oracle import synth
    sd = synth.clip_state_dict(111)
    ia, _ = synth.adapter_state_dicts(111)
    vp = {k: torch.from_numpy(v).to(dev) for k, v in sd.items() if k.startswith("visual.")}
    eng = VisualEngine(vp, {k: torch.from_numpy(v).to(dev) for k, v in ia.items()}, dtype=torch.float16)
    g = torch.Generator(device=dev).manual_seed(5)
    xs = torch.randn(3, 3, 336, 336, device=dev, generator=g)
    T = torch.nn.functional.normalize(torch.randn(768, 2, device=dev, generator=g), dim=0).contiguous()
    predict = lambda x, t=T: eng.predict(x, t, "Industrial")  # noqa: E731
    _, s_local, s_all, m_all = sharded_step(predict, xs, T, 3, gather_maps=True)
    assert m_all is not None and m_all.shape[0] == 3
    r = verify_gather(lambda x: predict(x)[1], lambda a, b: xs[a:b], s_all, s_local, 3)
    assert r["backend"] == "nccl" and r["world"] == 1
    assert r["own_slice_verified"] and r["gather_verified"], r
