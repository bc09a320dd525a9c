"""The data-parallel path of config C3 (images sharded over ranks, one process per GPU,
scores all-gathered) driven through the REAL HIP engine in two processes.

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so the
bench's rehearsal mode puts both ranks on cuda:0 over gloo: the same self-launch
(torch.distributed.run as a child), shard_range slices of one seeded global batch, the
per-step all-gather, max-over-ranks timing and the post-hoc self-check
(parallel.verify_gather: every rank finds its own scores in the gathered vector, rank 0
recomputes the other rank's shard with an eager one-stream predict and compares bit for
bit) -- on VisualEngine outputs, not a CPU stand-in (tests/test_distributed_gloo.py).
Reference: the per-batch loop being sharded, test.py:53-99.

The bench is started as a FRESH child process (never an exec of this test process, which
has initialised the GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_bench_two_ranks_real_engine(dev):
    env = dict(os.environ, AACLIP_BENCH_REHEARSAL="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-c5", "--no-modes", "--no-roofline", "--cpu-seconds", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    print({k: line[k] for k in ("value", "n_gpus", "ms_per_step")}, line["distributed"])
    assert line["n_gpus"] == 2
    assert line["config"]["global_batch"] == 64
    d = line["distributed"]
    assert d["world"] == 2 and d["backend"] == "gloo"
    assert d["gather_verified"] and d["own_slice_verified"], d
    assert d["checked_shard"]["rank"] == 1 and d["checked_shard"]["images"] == [32, 64]
    assert line["step_outputs_verified"]["finite"] and line["step_outputs_verified"]["equal_to_one_stream_eager"]
    assert line["parity_gate"] is True, line.get("parity_gate_failed")


@pytest.mark.timeout(900)
def test_bench_c3_partition_eight_ranks_real_engine(dev):
    """Config C3's exact partition through the real engine: 8 ranks x 32 images = a global
    batch of 256 (shard_range: rank r owns [32 r, 32 r + 32)), the per-step score
    all-gather, max-over-ranks timing, the post-hoc self-check (rank 0 recomputes rank 7's
    shard [224, 256) eagerly and compares bit for bit) and rank 0's timed-step check
    against the CPU oracle with the parity gate. All 8 ranks share cuda:0 over gloo (RCCL
    refuses two ranks on one device): a plumbing check of the N = 8 launch, not a scaling
    number. Started as a fresh child process. Reference: test.py:53-99."""
    env = dict(os.environ, AACLIP_BENCH_REHEARSAL="1", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "8", "--batch", "32", "--steps", "2",
           "--warmup", "1", "--no-c5", "--no-modes", "--no-roofline", "--cpu-seconds", "0", "--streams", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=840)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    print({k: line[k] for k in ("value", "n_gpus", "ms_per_step")}, line["distributed"], line["timed_step_vs_oracle"])
    assert line["n_gpus"] == 8
    assert line["config"]["global_batch"] == 256 and line["config"]["per_gpu_batch"] == 32
    d = line["distributed"]
    assert d["world"] == 8 and d["backend"] == "gloo"
    assert d["gather_verified"] and d["own_slice_verified"], d
    assert d["checked_shard"] == {"rank": 7, "images": [224, 256], "checked_by": 0}
    assert len(d["ms_per_step_per_rank"]) == 8 and max(d["ms_per_step_per_rank"]) == line["ms_per_step"]
    assert line["step_outputs_verified"]["finite"] and line["step_outputs_verified"]["equal_to_one_stream_eager"]
    assert line["parity_gate"] is True and "timed_step_vs_oracle" in line["parity_gate_checked"]


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(900)
def test_harness_two_ranks_real_engine(dev, tmp_path):
    """The harness's multi-rank path (aa-clip_amd/test.py under torchrun: each class's images
    sharded by shard_range, per-rank predict on the real engine, maps / scores / masks /
    labels / names gathered onto rank 0, rank-0 device metrics_eval) against the same harness
    in one process. 7 images per class over 2 ranks (an uneven 4 + 3 shard), 15 classes
    (C4's synthetic_mvtec flow). Both runs are FRESH child processes; the rehearsal puts
    both ranks on cuda:0 over gloo (AACLIP_REHEARSAL=1). Reference: test.py:53-99,211-249."""
    script = os.path.join(ROOT, "aa-clip_amd", "test.py")
    common = ["--dataset", "synthetic_mvtec", "--allow_random_init", "--synthetic_n", "7", "--img_size", "336",
              "--compute_dtype", "fp16"]
    one, two = tmp_path / "single.json", tmp_path / "two_ranks.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-u", script, *common, "--save_path", str(tmp_path / "s1"),
                        "--results_json", str(one)], cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    env2 = dict(env, AACLIP_REHEARSAL="1")
    r = subprocess.run([sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script, *common,
                        "--save_path", str(tmp_path / "s2"), "--results_json", str(two)],
                       cwd=ROOT, env=env2, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    a, b = json.loads(one.read_text()), json.loads(two.read_text())
    assert a["world"] == 1 and b["world"] == 2
    assert len(a["rows"]) == 16  # 15 classes + the average row
    print(b["rows"][-1])
    assert a["rows"] == b["rows"]  # every per-class pixel / image AUROC and AP, exactly
