# round-4 pass: the r04a suite/bench/A-B, then the attention variant-5 experiment
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r04a.sh r04a || exit $?
bash tools/gpu_attn5.sh attn5
