#!/bin/bash
# epilogue store contention probe (tools/store_contention.py)
set -o pipefail
mkdir -p gpurun_out/r04i
timeout -k 10 300 python -u tools/store_contention.py > gpurun_out/r04i/store_contention.txt 2>&1
