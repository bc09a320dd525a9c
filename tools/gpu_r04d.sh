# round-4: attention variants 5-7 vs 3, GEMM L2 PMC table, quick-gelu bf16 flip count
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04d
timeout -k 10 200 python -u -m pytest tests/test_e2e_gpu.py -m gpu -q -s -k "quick_gelu" --timeout 150 \
  --timeout-method thread > gpurun_out/r04d/quick.log 2>&1 || { tail -20 gpurun_out/r04d/quick.log; exit 1; }
grep -E "flips" gpurun_out/r04d/quick.log
bash tools/gpu_attn5.sh attn6 || exit $?
cd /tmp && bash $R/tools/prof_pmc_l2.sh $R/gpurun_out/l2
