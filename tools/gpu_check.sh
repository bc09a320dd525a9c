# GPU box: GPU test suite, then the default bench line; stops after any fault / abort / timeout.
# usage: bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc2=$?
tail -c 3000 $OUT/bench.json; tail -5 $OUT/bench.err
exit $(( rc2 != 0 ? rc2 : rc ))
