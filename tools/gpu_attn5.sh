# attention variant 5 (32x32 pipelined) vs the default 3: tests, isolated timing, whole-step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-attn5}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "attention" --timeout 120 \
  --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 200 python -u tools/attn_variants.py --variants 3,5,6,7 --seqs 577,1025 --rounds 3 > $OUT/iso_bf16.txt 2>&1 || exit 1
cat $OUT/iso_bf16.txt
timeout -k 10 200 python -u tools/attn_variants.py --variants 3,6 --seqs 577 --rounds 2 --dtype fp16 > $OUT/iso_fp16.txt 2>&1 || exit 1
cat $OUT/iso_fp16.txt
ROUNDS="1 2" bash tools/step_ab.sh "--attn-variant 3" "--attn-variant 6" "--attn-variant 7" 2>&1 | tee $OUT/step_ab.txt
