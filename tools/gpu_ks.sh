# GPU box: split-K c_proj checks + in-step A/B. usage: bash tools/gpu_ks.sh TAG [arms...]
set -o pipefail
TAG=${1:-ks}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -q -x --timeout 300 --timeout-method thread \
  -k "ksplit or tune_gemm or fp8mx" > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u tools/step_arms.py "$@" > $OUT/arms.log 2>&1 || { echo arms failed; tail -20 $OUT/arms.log; exit 4; }
cat $OUT/arms.log
timeout -k 10 200 python -u tools/ksplit_bench.py > $OUT/ksplit_bench.log 2>&1 || { echo kbench failed; tail -20 $OUT/ksplit_bench.log; exit 5; }
cat $OUT/ksplit_bench.log
