"""Kernel micro-benchmark: times the per-block kernels of the C2 workload
(B=32, 577 tokens) in isolation with HIP events (random bf16 operands).

    python tools/kbench.py [--reps 20] [--only gemm|attn|rows]
Used for A/B work on the kernels and as the command profiled by rocprofv3 --pmc.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aa-clip_amd"))

import torch  # noqa: E402

from aaclip import ops  # noqa: E402


def timeit(fn, reps):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    fn()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--variants", default="0", help="comma list of GEMM variants, A/B interleaved")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--shapes", default="qkv,out,fc,proj,adapter", help="GEMM shapes to run")
    ap.add_argument("--map", action="store_true", help="also run the anomaly-map stream kernel (C2 sizes)")
    ap.add_argument("--fp8", action="store_true", help="also time the fp8 GEMM (+ the row quantisation of A)")
    ap.add_argument("--mx", action="store_true", help="also time the fp8 MX GEMM per --variants (0 vs 5)")
    ap.add_argument("--tokens", type=int, default=577, help="tokens per image (577 @336 px, 1025 @448 px)")
    ap.add_argument("--torch", action="store_true",
                    help="also time torch (hipBLASLt) on the same GEMM shapes, for comparison only")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B, n, W = args.batch, args.tokens, 1024
    R = B * n
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s, std=1.0: (torch.randn(*s, device=dev, generator=g) * std)  # noqa: E731
    h = rnd(R, W).bfloat16()
    x = rnd(R, W)
    res = {}
    if args.only in ("", "gemm"):
        shapes = {"qkv": (3 * W, W, dict(bias=True)), "out": (W, W, dict(bias=True, resid=True)),
                  "fc": (4 * W, W, dict(bias=True, gelu=True)), "proj": (W, 4 * W, dict(bias=True, resid=True)),
                  "adapter": (W, W, dict(leaky=True))}
        from aaclip import _lib
        variants = [int(v) for v in args.variants.split(",")]
        data = {}
        shapes = {n: v for n, v in shapes.items() if n in args.shapes.split(",")}
        for name, (N, K, kw) in shapes.items():
            a = rnd(R, K).bfloat16()
            w = rnd(N, K, std=K ** -0.5).bfloat16()
            bias = rnd(N, std=0.02)
            out = torch.empty(R, N, device=dev, dtype=torch.float32 if (kw.get("resid") or kw.get("leaky")) else torch.bfloat16)
            data[name] = (N, K, kw, a, w, bias, out)
        for rnd_i in range(args.rounds):
            for v in variants:
                _lib.call("aaclip_set_gemm_variant", v)
                for name, (N, K, kw, a, w, bias, out) in data.items():
                    f = lambda: ops.gemm(a, w, out, bias=bias if kw.get("bias") else None, gelu=kw.get("gelu", False),  # noqa: E731
                                         leaky=kw.get("leaky", False), residual=out if kw.get("resid") else None)
                    ms = timeit(f, args.reps)
                    key = name if len(variants) == 1 else f"{name}/v{v}"
                    prev = res.get(key)
                    if prev is None or ms < prev[0]:
                        res[key] = (ms, 2.0 * R * N * K / ms / 1e9)
        _lib.call("aaclip_set_gemm_variant", 0)
        if args.fp8:
            FP8 = torch.float8_e4m3fn
            for name, (N, K, kw, a, w, bias, out) in data.items():
                a8 = torch.empty(R, K, device=dev, dtype=FP8)
                sa = torch.empty(R, device=dev)
                ops.quant_fp8_rows(a, a8, sa)
                sw = (w.float().abs().amax(1) / 448).contiguous()
                w8 = (w.float() / sw[:, None]).to(FP8)
                f = lambda: ops.gemm_fp8(a8, sa, w8, sw, out, bias=bias if kw.get("bias") else None,  # noqa: E731
                                         gelu=kw.get("gelu", False), leaky=kw.get("leaky", False),
                                         residual=out if kw.get("resid") else None)
                ms = timeit(f, args.reps)
                res[f"{name}/fp8"] = (ms, 2.0 * R * N * K / ms / 1e9)
                ms = timeit(lambda: ops.quant_fp8_rows(a, a8, sa), args.reps)
                res[f"{name}/quantA"] = (ms, R * K * 3 / ms / 1e9)
        if args.mx:
            FP8 = torch.float8_e4m3fn
            mx = {}
            for name, (N, K, kw, a, w, bias, out) in data.items():
                a8 = torch.empty(R, K, device=dev, dtype=FP8)
                asc = ops.mx_scales(R, K, dev)
                ops.quant_fp8_mx(a.float(), a8, asc)
                sw = (w.float().abs().amax(1) / 448).contiguous()
                w8 = (w.float() / sw[:, None]).to(FP8)
                if kw.get("gelu"):  # c_fc writes fp8 MX for c_proj
                    o8, osc = torch.empty(R, N, device=dev, dtype=FP8), ops.mx_scales(R, N, dev)
                else:
                    o8, osc = out, None
                mx[name] = (N, K, kw, a8, asc, w8, sw, bias, o8, osc)
            for rnd_i in range(args.rounds):
                for v in variants:
                    _lib.call("aaclip_set_gemm_variant", v)
                    for name, (N, K, kw, a8, asc, w8, sw, bias, o8, osc) in mx.items():
                        f = lambda: ops.gemm_fp8mx(a8, asc, w8, sw, o8, out_sc=osc,  # noqa: E731
                                                   bias=bias if kw.get("bias") else None, gelu=kw.get("gelu", False),
                                                   leaky=kw.get("leaky", False),
                                                   residual=o8 if kw.get("resid") else None)
                        ms = timeit(f, args.reps)
                        key = f"{name}/mx/v{v}"
                        prev = res.get(key)
                        if prev is None or ms < prev[0]:
                            res[key] = (ms, 2.0 * R * N * K / ms / 1e9)
            _lib.call("aaclip_set_gemm_variant", 0)
        if args.torch:  # library comparison: linear (+bias) -> epilogue in torch ops
            F = torch.nn.functional
            for name, (N, K, kw, a, w, bias, out) in data.items():
                bb = bias.bfloat16() if kw.get("bias") else None
                x32 = torch.randn(R, N, device=dev) if kw.get("resid") else None
                f0 = lambda: F.linear(a, w, bb)  # noqa: E731
                if kw.get("gelu"):
                    f = lambda: F.gelu(F.linear(a, w, bb))  # noqa: E731
                elif kw.get("resid"):
                    f = lambda: x32.add_(F.linear(a, w, bb))  # noqa: E731
                elif kw.get("leaky"):
                    f = lambda: F.leaky_relu(F.linear(a, w))  # noqa: E731
                else:
                    f = f0
                for key, fn in ((f"{name}/torch-gemm", f0), (f"{name}/torch-full", f)):
                    ms = timeit(fn, args.reps)
                    res[key] = (ms, 2.0 * R * N * K / ms / 1e9)
    if args.only in ("", "attn"):
        qkv = rnd(R, 3 * W).bfloat16()
        o = torch.empty(R, W, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: ops.attention(qkv, o, B, n, 16), args.reps)
        res["attn"] = (ms, 4.0 * B * n * n * W / ms / 1e9)
    if args.map:
        P = B * 576
        seg = rnd(P, 5 * 768)
        levels = [seg[:, j * 768:(j + 1) * 768] for j in range(4)]
        T = torch.nn.functional.normalize(rnd(768, 2), dim=0).contiguous()
        grid = torch.empty(P, device=dev)
        ms = timeit(lambda: ops.patch_scores(levels, T, grid), args.reps)
        res["patch_scores"] = (ms, (4 * P * 768 * 4 + P * 4) / ms / 1e6)
        S = 14 * 24
        amap = torch.empty(B, S, S, device=dev)  # both stages: patch scores + blur/upsample
        ms = timeit(lambda: ops.anomaly_map(levels, T, amap, grid, g=24, ksize=7, sigma=1.0), args.reps)
        res["anomaly_map"] = (ms, (4 * P * 768 * 4 + B * S * S * 4) / ms / 1e6)
        # the predict() form since round 4: map + image score from the projection GEMMs'
        # per-(row, 32-column) partials (4 levels + det, 24 groups of {||v||^2, v.t0, v.t1, 0})
        part = torch.rand(P, 5 * 4 * ops.SCORE_GROUPS, device=dev, generator=g) + 0.5
        det_ws, score = torch.empty(P, device=dev), torch.empty(B, device=dev)
        ms = timeit(lambda: ops.anomaly_map_partials(part, 4, amap, grid, g=24, ksize=7, sigma=1.0, det_ws=det_ws,
                                                     score=score), args.reps)
        res["anomaly_map_partials"] = (ms, (part.numel() * 4 + B * S * S * 4 + 2 * P * 4) / ms / 1e6)
    if args.only == "prep":  # device preprocessing: B decoded 1024x1024 RGB -> fp32 [B,3,S,S] (+ masks)
        from aaclip.preprocess import Preprocessor
        S = 336 if args.tokens == 577 else 448
        for H in (900, 1024):
            u8 = torch.randint(0, 256, (B, H, H, 3), device=dev, dtype=torch.uint8)
            m8 = (torch.rand(B, H, H, device=dev) < 0.1).to(torch.uint8)
            pp = Preprocessor(S)
            out = torch.empty(B, 3, S, S, device=dev)
            mo = torch.empty(B, 1, S, S, device=dev)
            ms = timeit(lambda: pp.images(u8, out), args.reps)
            res[f"prep{H}"] = (ms, (u8.numel() + out.numel() * 4) / ms / 1e6)
            ms = timeit(lambda: pp.masks(m8, mo), args.reps)
            res[f"mask{H}"] = (ms, (B * S * S * (1 + 4)) / ms / 1e6)
    if args.only in ("", "rows"):
        lw, lb = rnd(W), rnd(W)
        ms = timeit(lambda: ops.layernorm(x, lw, lb, h), args.reps)
        res["layernorm"] = (ms, (R * W * 6) / ms / 1e6)
    for k, (ms, rate) in res.items():
        unit = "GB/s" if k in ("layernorm", "patch_scores", "anomaly_map", "anomaly_map_partials") or k.endswith("quantA") or k[:4] in ("prep", "mask") \
            else "TFLOP/s"
        print(f"{k:10s} {ms * 1e3:9.1f} us  {rate:8.1f} {unit}")


if __name__ == "__main__":
    main()
