#!/bin/bash
# 8-phase GEMM: each phase's LDS-DMA issued before its ds_reads (guide: stage first) vs after
set -o pipefail
mkdir -p gpurun_out/r04aa
AACLIP_LIB=ab/libaaclip_dmafirst.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m gpu tests/test_kernels_gpu.py -k gemm > gpurun_out/r04aa/pytest.log 2>&1 || { tail -20 gpurun_out/r04aa/pytest.log; exit 1; }
tail -1 gpurun_out/r04aa/pytest.log
bash tools/lib_ab.sh ab/libaaclip_base.so ab/libaaclip_dmafirst.so > gpurun_out/r04aa/lib_ab.txt 2>&1
cat gpurun_out/r04aa/lib_ab.txt
