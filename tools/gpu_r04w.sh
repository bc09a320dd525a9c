#!/bin/bash
# LayerNorm weight / bias rows staged in LDS per workgroup: library A/B of the C2 step vs HEAD
set -o pipefail
mkdir -p gpurun_out/r04w
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so > gpurun_out/r04w/lib_ab.txt 2>&1
cat gpurun_out/r04w/lib_ab.txt
