#!/bin/bash
# persistent 8-phase GEMM with two tiles per workgroup (grid = tiles / 2: the second tile's
# prologue under the first's epilogue, dynamic workgroup placement kept) vs the default
set -o pipefail
mkdir -p gpurun_out/r04t
AACLIP_LIB=ab/libaaclip_p2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm" > gpurun_out/r04t/pytest.log 2>&1 || { tail -20 gpurun_out/r04t/pytest.log; exit 1; }
tail -1 gpurun_out/r04t/pytest.log
for r in 1 2 3; do
  for arm in "ab/libaaclip_base.so 0" "ab/libaaclip_p2.so 5"; do
    set -- $arm
    AACLIP_LIB=$1 timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-roofline --cpu-seconds 0 --no-modes \
      --no-c5 --gemm-variant $2 > gpurun_out/r04t/b.json 2>/dev/null || exit 1
    echo "round $r $1 v$2 $(python -c "import json;d=json.load(open('gpurun_out/r04t/b.json'));print(d['value'], d['ms_per_step'])")"
  done
done | tee gpurun_out/r04t/ab.txt
