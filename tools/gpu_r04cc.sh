#!/bin/bash
# quad-coalesced 8-phase epilogue (per-wave LDS transposition): GEMM kernel suite, the
# in-kernel epilogue stamps, then the whole-step library A/B against the HEAD build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04cc_kernels.txt 2>&1 || { tail -30 gpurun_out/r04cc_kernels.txt; exit 1; }
tail -3 gpurun_out/r04cc_kernels.txt
timeout -k 10 120 python tools/epi_stamps.py --M 9232,18464 > gpurun_out/r04cc_stamps.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04cc_stamps.txt
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so | tee gpurun_out/r04cc_ab.txt
