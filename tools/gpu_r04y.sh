#!/bin/bash
# fp8 MX 8-phase GEMM: tile bias staged in LDS (as the bf16 kernel): fp8 tests, then C5 A/B vs HEAD
set -o pipefail
mkdir -p gpurun_out/r04y
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_e2e_gpu.py -k "fp8 or mx or c5 or C5 or deferred" \
  > gpurun_out/r04y/pytest.log 2>&1 || { tail -30 gpurun_out/r04y/pytest.log; exit 1; }
tail -1 gpurun_out/r04y/pytest.log
for r in 1 2 3; do
  for lib in ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so; do
    echo "round $r $lib c5: $(AACLIP_LIB=$lib timeout -k 10 200 python tools/c5_ab.py 2>/dev/null | tail -1)" \
      | tee -a gpurun_out/r04y/c5_ab.txt
  done
done
