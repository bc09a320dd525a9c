"""One C5 timing line for the library AACLIP_LIB points at (bench.c5_leg: fp8 on the MLP,
fp8 on every block GEMM, bf16; graphed two-stream predict at 448 px, batch 32), for
interleaved library A/B rounds (tools/gpu_ab.sh).
usage: AACLIP_LIB=path python tools/c5_ab.py [--steps 10]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-clip_amd")]
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    out = bench.c5_leg(torch.device("cuda:0"), a.steps, 2, 2)
    print(f"fp8 {out['fp8']['images_per_sec']} fp8_all {out['fp8_all']['images_per_sec']} "
          f"bf16 {out['bf16']['images_per_sec']} fp8_gemm_us {out['fp8_gemm_roofline']['avg_launch_us']}")


if __name__ == "__main__":
    main()
