# Round 4 first GPU pass: bf16 flip counts (-s), the GPU suite, the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04a}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py -m gpu -q -s -k "bf16_parity or 518" --timeout 250 \
  --timeout-method thread > $OUT/flips.log 2>&1 || { echo "flip tests rc=$?"; tail -20 $OUT/flips.log; exit 1; }
grep -E "bf16:|flips" $OUT/flips.log | head
bash tools/gpu_check.sh ${1:-r04a}
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/engine_ab.py base= defer=defer_resid:1 > $OUT/ab_defer.txt 2>&1; tail -4 $OUT/ab_defer.txt
timeout -k 10 300 python -u tools/engine_ab.py base= defer=defer_resid:1 --streams 1 > $OUT/ab_defer_1s.txt 2>&1; tail -4 $OUT/ab_defer_1s.txt
