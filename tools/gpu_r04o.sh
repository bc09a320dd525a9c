#!/bin/bash
# 8-phase GEMM priority A/B: HEAD (setprio 1/0 around each MFMA cluster), young wave row kept
# at prio 1 after its clusters, static prio 1 for the young row with no per-cluster flips
set -o pipefail
mkdir -p gpurun_out/r04o
bash tools/lib_ab.sh ab/libaaclip_base.so ab/libaaclip_prio.so ab/libaaclip_prio2.so > gpurun_out/r04o/lib_ab.txt 2>&1
cat gpurun_out/r04o/lib_ab.txt
