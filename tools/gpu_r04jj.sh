#!/bin/bash
# round-4 final tree (quad-coalesced GEMM epilogues): GPU suite + smoke + bench + C4, the
# rocprofv3 kernel trace + stats of the default bench command, then the PMC traffic passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r04_final.sh || exit $?
bash tools/gpu_r04r.sh || exit $?
