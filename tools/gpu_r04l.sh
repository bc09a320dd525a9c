#!/bin/bash
# 8-phase GEMM back to 224 VGPRs (scores path in its own instantiation): GEMM / map / e2e
# tests, then library A/B of the whole C2 step against the 226-VGPR build
set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_map_partials_gpu.py tests/test_e2e_gpu.py \
  > gpurun_out/r04l/pytest.log 2>&1 || { tail -30 gpurun_out/r04l/pytest.log; exit 1; }
tail -2 gpurun_out/r04l/pytest.log
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so > gpurun_out/r04l/lib_ab.txt 2>&1
cat gpurun_out/r04l/lib_ab.txt
