#!/bin/bash
# quad-coalesced epilogue on the fp8 MX 8-phase kernel (c_fc -> e4m3 + block scales,
# c_proj fp32 + residual): fp8 / GEMM suites, then C5 (HEAD / this build), 3 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ii
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp8_gpu.py \
  tests/test_kernels_gpu.py > gpurun_out/r04ii/pytest.log 2>&1 || { tail -30 gpurun_out/r04ii/pytest.log; exit 1; }
tail -1 gpurun_out/r04ii/pytest.log
for r in 1 2 3; do
  for lib in ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so; do
    echo "round $r $lib c5: $(AACLIP_LIB=$lib timeout -k 10 200 python tools/c5_ab.py 2>/dev/null | tail -1)" \
      | tee -a gpurun_out/r04ii/c5_ab.txt
  done
done
