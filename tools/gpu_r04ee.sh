#!/bin/bash
# residual-by-LDS-DMA 8-phase epilogue (ab/libaaclip_dma.so): GEMM kernel suite and
# epilogue stamps on it, then the whole-step A/B: HEAD build / quad-coalesced epilogue
# (in-tree) / + residual DMA
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AACLIP_LIB=ab/libaaclip_dma.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r04ee_kernels.txt 2>&1 || { tail -30 gpurun_out/r04ee_kernels.txt; exit 1; }
tail -2 gpurun_out/r04ee_kernels.txt
AACLIP_LIB=ab/libaaclip_dma.so timeout -k 10 120 python tools/epi_stamps.py --M 9232,18464 > gpurun_out/r04ee_stamps.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04ee_stamps.txt | grep -A3 "^out"
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so ab/libaaclip_dma.so | tee gpurun_out/r04ee_ab.txt
