#!/bin/bash
# attention: static prio 1 for every other workgroup of an XCD (3 share a CU) vs none;
# then the persistent 8-phase GEMM family in the step
set -o pipefail
mkdir -p gpurun_out/r04q
ATTN=1 bash tools/lib_ab.sh ab/libaaclip_base.so ab/libaaclip_attnprio.so > gpurun_out/r04q/lib_ab.txt 2>&1
cat gpurun_out/r04q/lib_ab.txt
# persistent 8-phase GEMM (family 5) vs the default dispatch in the step, current kernel
ROUNDS="1 2 3" bash tools/step_ab.sh "--gemm-variant 0" "--gemm-variant 5" > gpurun_out/r04q/persist_ab.txt 2>&1
cat gpurun_out/r04q/persist_ab.txt
