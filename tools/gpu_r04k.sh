#!/bin/bash
# per-CU store throughput by store-instruction shape (tools/store_bench.hip)
set -o pipefail
mkdir -p gpurun_out/r04k
timeout -k 10 120 ./tools/_store_bench > gpurun_out/r04k/store_bench.txt 2>&1
