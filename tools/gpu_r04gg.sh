#!/bin/bash
# whole-step A/B, 4 interleaved rounds: HEAD build / quad-coalesced epilogue with the
# run-time-flag epilogues routed to the 320x256 kernel (in-tree) / with them kept in the
# 8-phase kernel's LDS epilogue (250 VGPRs)
set -o pipefail
cd $GRAFT_REPO_ROOT
ROUNDS=4 bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so ab/libaaclip_v250.so \
  | tee gpurun_out/r04gg_ab.txt
