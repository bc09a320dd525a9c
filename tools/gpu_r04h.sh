# chunk stagger A/B (whole two-stream step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r04h
timeout -k 10 400 python -u tools/engine_ab.py base= s1=stagger:1 s2=stagger:2 s4=stagger:4 s8=stagger:8 --rounds 3 \
  > gpurun_out/r04h/ab_stagger.txt 2>&1; rc=$?
tail -7 gpurun_out/r04h/ab_stagger.txt; exit $rc
