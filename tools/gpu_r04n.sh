#!/bin/bash
# LDS-staged residual epilogue of the 8-phase GEMM: GEMM (families bit-identical incl. aux),
# map and e2e tests, the epilogue stamps, then library A/B of the C2 step against HEAD
set -o pipefail
mkdir -p gpurun_out/r04n
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_map_partials_gpu.py tests/test_e2e_gpu.py \
  > gpurun_out/r04n/pytest.log 2>&1 || { tail -30 gpurun_out/r04n/pytest.log; exit 1; }
tail -2 gpurun_out/r04n/pytest.log
timeout -k 10 200 python -u tools/epi_stamps.py > gpurun_out/r04n/epi_stamps.txt 2>&1 || exit 1
cat gpurun_out/r04n/epi_stamps.txt
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so > gpurun_out/r04n/lib_ab.txt 2>&1
cat gpurun_out/r04n/lib_ab.txt
