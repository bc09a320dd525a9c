# GPU box, round check: full GPU suite, smoke(), the default bench line (parity-gated),
# then rocprofv3 kernel trace + stats of the same bench command (per-grid summary).
# Stops after any fault / abort / timeout. usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 4; }
bash tools/prof_bench.sh gpurun_out/$TAG/prof > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $OUT/prof.log; exit 5; }
exit $rc
