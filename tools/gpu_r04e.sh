# round-4: chunk-stream priority A/B (whole two-stream step, interleaved rounds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04e
timeout -k 10 300 python -u tools/engine_ab.py base= prio=stream_prio:1 --rounds 5 > gpurun_out/r04e/ab_prio.txt 2>&1; rc=$?
tail -4 gpurun_out/r04e/ab_prio.txt; exit $rc
