#!/bin/bash
# attention key-tail K/V rows staged in LDS by a prologue DMA: attention / e2e tests, then
# library A/B (attention alone + C2 step) against HEAD
set -o pipefail
mkdir -p gpurun_out/r04s
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_e2e_gpu.py -k "attention or attn or golden or e2e or parity" \
  > gpurun_out/r04s/pytest.log 2>&1 || { tail -30 gpurun_out/r04s/pytest.log; exit 1; }
tail -1 gpurun_out/r04s/pytest.log
ATTN=1 bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so > gpurun_out/r04s/lib_ab.txt 2>&1
cat gpurun_out/r04s/lib_ab.txt
