#!/bin/bash
# concurrent chunks: the 8-phase tile for every N % 256 block / projection GEMM (also the
# 108-tile N = 768 level projections, now 128x128 by the small-launch rule) vs HEAD
set -o pipefail
mkdir -p gpurun_out/r04z
bash tools/lib_ab.sh ab/libaaclip_base.so ab/libaaclip_conc8.so > gpurun_out/r04z/lib_ab.txt 2>&1
cat gpurun_out/r04z/lib_ab.txt
