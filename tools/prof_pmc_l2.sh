#!/bin/bash
# PMC passes over tools/l2_reuse.py run (one counter group per rocprofv3 run, kernel-trace
# only), then the per-(shape, group height) traffic table.
# usage (GPU box): bash tools/prof_pmc_l2.sh gpurun_out/l2
set -o pipefail
OUT=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$OUT"
groups=(
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"
)
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc$i" -o run -- python3 $R/tools/l2_reuse.py run \
    > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 "$OUT/pmc$i.log"; exit 1; }
  i=$((i+1))
done
python3 $R/tools/l2_reuse.py summarize "$OUT" --out "$OUT/l2_reuse.json"
