#!/bin/bash
# whole-step A/B, 4 interleaved rounds: HEAD build / quad-coalesced epilogue at 216 VGPRs
# (in-tree) / its first form at 250 VGPRs / + residual by LDS-DMA (206 VGPRs)
set -o pipefail
cd $GRAFT_REPO_ROOT
ROUNDS=4 bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so ab/libaaclip_v250.so \
  ab/libaaclip_dma.so | tee gpurun_out/r04ff_ab.txt
