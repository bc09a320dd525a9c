# round-4 final-tree check: GPU suite + smoke + bench + C4 (tools/gpu_final.sh), then the
# rocprofv3 kernel trace + stats of the default bench command (tools/prof_bench.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_final.sh r04_final || exit $?
bash tools/prof_bench.sh gpurun_out/r04_prof
