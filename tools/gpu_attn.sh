# GPU box: attention variant numerics + isolated + in-step A/B. usage: bash tools/gpu_attn.sh TAG VARIANTS ARMS...
set -o pipefail
TAG=${1:-attn}; VARS=${2:-3,4,5}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread \
  -k "attention" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/attn_variants.py --variants $VARS --rounds 3 --seqs 577,1025 > $OUT/attn_variants.log 2>&1 || { echo variants failed; tail -20 $OUT/attn_variants.log; exit 4; }
cat $OUT/attn_variants.log
timeout -k 10 300 python -u tools/step_arms.py "$@" > $OUT/arms.log 2>&1 || { echo arms failed; tail -20 $OUT/arms.log; exit 5; }
cat $OUT/arms.log
