# round-4: attention variant 5 experiment, deferred-residual engine A/B, GEMM L2 PMC table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04c
timeout -k 10 300 python -u tools/engine_ab.py base= defer=defer_resid:1 > gpurun_out/r04c/ab_defer.txt 2>&1; rc=$?
tail -4 gpurun_out/r04c/ab_defer.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/engine_ab.py base= defer=defer_resid:1 --streams 1 > gpurun_out/r04c/ab_defer_1s.txt 2>&1; rc=$?
tail -3 gpurun_out/r04c/ab_defer_1s.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_attn5.sh attn5 || exit $?
cd /tmp && bash $R/tools/prof_pmc_l2.sh $R/gpurun_out/l2
