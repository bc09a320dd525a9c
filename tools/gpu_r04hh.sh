#!/bin/bash
# quad-coalesced 8-phase epilogue, final form: full GPU suite + smoke + bench + C4
# (tools/gpu_final.sh), then the in-kernel epilogue stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh r04_quad || exit $?
timeout -k 10 120 python tools/epi_stamps.py --M 1024,5376,9232,18464 > gpurun_out/r04_quad/stamps.txt 2>&1 || exit 6
grep -v amdgpu.ids gpurun_out/r04_quad/stamps.txt
python -c "import json;d=json.load(open('gpurun_out/r04_quad/bench.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
