#!/bin/bash
# whole-step A/B: HEAD build / quad-coalesced 8-phase epilogue (216 VGPRs, run-time-flag
# epilogues routed to the 320x256 kernel) / the same with the run-time-flag path kept in
# the 8-phase kernel (224 VGPRs)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so ab/libaaclip_v224gen.so | tee gpurun_out/r04dd_ab.txt
