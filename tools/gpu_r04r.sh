#!/bin/bash
# round-4 final-tree PMC passes for the bench roofline traffic: block GEMMs (QKV, c_fc at
# M = 18464 on the 8-phase kernel) and the predict() anomaly map (partials form)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
bash $R/tools/prof_pmc.sh $R/gpurun_out/r04_pmc -- python3 $R/tools/kbench.py --only gemm --shapes qkv,fc --map --reps 5 || exit 1
cd $R
python tools/pmc_summary.py gpurun_out/r04_pmc --out gpurun_out/r04_pmc/summary.json \
  --traffic-out gpurun_out/r04_pmc/pmc_traffic.json > gpurun_out/r04_pmc/summary.txt 2>&1 || exit 1
cat gpurun_out/r04_pmc/summary.txt gpurun_out/r04_pmc/pmc_traffic.json
