# attention 32x32 kernel with conflict-free swizzles: tests, isolated timing, PMC, step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04g
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "attention" --timeout 120 \
  --timeout-method thread > gpurun_out/r04g/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04g/tests.log; [ $rc -ne 0 ] && { grep -E "assert|FAILED" gpurun_out/r04g/tests.log | head; exit $rc; }
timeout -k 10 200 python -u tools/attn_variants.py --variants 3,5,6 --seqs 577,1025 --rounds 3 > gpurun_out/r04g/iso.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r04g/iso.txt
bash tools/prof_pmc_attn.sh $R/gpurun_out/pmc_attn_v6b 6 577 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_attn_v6b --out gpurun_out/pmc_attn_v6b/summary.json | grep attn
ROUNDS="1 2" bash tools/step_ab.sh "--attn-variant 3" "--attn-variant 6" 2>&1 | tee gpurun_out/r04g/step_ab.txt
