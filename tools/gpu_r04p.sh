#!/bin/bash
# GEMM priority follow-up: C2 step (HEAD / static young-row prio / no prio at all), then C5
# (HEAD / bf16 kernel only / bf16 + fp8 MX kernel with the static priority)
set -o pipefail
mkdir -p gpurun_out/r04p
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "gemm" > gpurun_out/r04p/pytest.log 2>&1 || { tail -30 gpurun_out/r04p/pytest.log; exit 1; }
tail -1 gpurun_out/r04p/pytest.log
bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so ab/libaaclip_noprio.so \
  > gpurun_out/r04p/lib_ab.txt 2>&1 || { cat gpurun_out/r04p/lib_ab.txt; exit 1; }
cat gpurun_out/r04p/lib_ab.txt
for r in 1 2; do
  for lib in ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so ab/libaaclip_fp8prio.so; do
    echo "round $r $lib c5: $(AACLIP_LIB=$lib timeout -k 10 200 python tools/c5_ab.py 2>/dev/null | tail -1)" \
      | tee -a gpurun_out/r04p/c5_ab.txt
  done
done
