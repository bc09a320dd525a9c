#!/bin/bash
# tile bias staged in LDS for the 8-phase epilogue + 16-B attention output stores:
# GEMM / attention / map / e2e tests, then library A/B (HEAD, bias only, both) of the
# attention kernel alone and the whole C2 step
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_map_partials_gpu.py tests/test_e2e_gpu.py \
  > gpurun_out/r04m/pytest.log 2>&1 || { tail -30 gpurun_out/r04m/pytest.log; exit 1; }
tail -2 gpurun_out/r04m/pytest.log
ATTN=1 bash tools/lib_ab.sh ab/libaaclip_base.so ab/libaaclip_bias.so aa-clip_amd/aaclip/libaaclip_hip.so \
  > gpurun_out/r04m/lib_ab.txt 2>&1
cat gpurun_out/r04m/lib_ab.txt
