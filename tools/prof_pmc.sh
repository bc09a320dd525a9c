#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only; never
# combined with sys/runtime traces) over a command; CSVs under $OUT.
# usage: tools/prof_pmc.sh OUTDIR -- python tools/kbench.py --only gemm
set -o pipefail
OUT=$1; shift; [ "$1" == "--" ] && shift
export TMPDIR=/tmp
mkdir -p "$OUT"
groups=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
i=0
for g in "${groups[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc$i" -o run -- "$@" > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
  i=$((i+1))
done
echo "pmc ok"
