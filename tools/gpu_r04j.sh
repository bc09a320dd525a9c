#!/bin/bash
# epilogue s_memtime stamps (tools/epi_stamps.py) + GEMM family bit-identity test
set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 200 python -u tools/epi_stamps.py > gpurun_out/r04j/epi_stamps.txt 2>&1
