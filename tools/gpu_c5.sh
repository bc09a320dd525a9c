# GPU box: C5 per-op profile + chunking arms (fp8 and bf16). usage: bash tools/gpu_c5.sh TAG
set -o pipefail
TAG=${1:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/c5_profile.py --out $OUT/c5_profile.json > $OUT/c5_profile.log 2>&1 || { echo "profile rc=$?"; tail -5 $OUT/c5_profile.log; exit 3; }
timeout -k 10 300 python -u tools/chunk_arms.py --dtype fp8 16,16 15,17 14,18 15,15,2 > $OUT/chunks_fp8.log 2>&1 || { echo "fp8 arms rc=$?"; tail -5 $OUT/chunks_fp8.log; exit 4; }
timeout -k 10 300 python -u tools/chunk_arms.py --dtype bf16 16,16 15,17 14,18 15,15,2 > $OUT/chunks_bf16.log 2>&1 || { echo "bf16 arms rc=$?"; tail -5 $OUT/chunks_bf16.log; exit 5; }
grep -v amdgpu.ids $OUT/c5_profile.log $OUT/chunks_fp8.log $OUT/chunks_bf16.log
