#!/bin/bash
# determinism / deferred-residual identity of the LN change vs HEAD
set -o pipefail
for lib in ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so; do
  echo "== $lib"
  AACLIP_LIB=$lib timeout -k 10 200 python tools/det_check.py bf16 2>&1 | grep -v amdgpu.ids || exit 1
done
