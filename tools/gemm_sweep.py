"""GEMM shape sweep for the bf16 kernel families (A/B interleaved in one
process): separates main-loop efficiency (long K) from per-tile overheads
(short K) and tile quantisation (tiles vs 256 CUs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aa-clip_amd"))
import torch  # noqa: E402

from aaclip import _lib, ops  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from kbench import timeit  # noqa: E402

dev = torch.device("cuda:0")
shapes = [(18464, 3072, 1024), (18432, 3072, 1024), (16384, 4096, 1024), (16384, 4096, 4096),
          (8192, 8192, 8192), (4096, 4096, 4096), (18464, 1024, 4096), (18432, 2048, 4096), (65536, 1024, 1024)]
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,2").split(",")]
best = {}
g = torch.Generator(device=dev).manual_seed(0)
for rnd in range(2):
    for (M, N, K) in shapes:
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for v in variants:
            _lib.call("aaclip_set_gemm_variant", v)
            ms = timeit(lambda: ops.gemm(a, w, out), 10)
            k = (M, N, K, v)
            best[k] = min(best.get(k, 1e9), ms)
        del a, w, out
_lib.call("aaclip_set_gemm_variant", 0)
for (M, N, K, v), ms in sorted(best.items()):
    tiles = -(-M // 256) * (N // (256 if (v in (1, 2) and N % 256 == 0) else 128))
    print(f"M={M:6d} N={N:5d} K={K:5d} v{v}: {ms*1e3:8.1f} us {2*M*N*K/ms/1e9:7.1f} TF/s  tiles={tiles} ({tiles/256:.2f} waves)")
