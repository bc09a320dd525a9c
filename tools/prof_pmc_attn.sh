#!/bin/bash
# PMC passes over the attention kernel (tools/attn_variants.py --eager, one variant
# and sequence length per run): wave-state split (parked / issue-stalled / active),
# LDS conflicts, MFMA busy. usage: tools/prof_pmc_attn.sh OUTDIR VARIANT [SEQ]
set -o pipefail
OUT=$1; VAR=$2; SEQ=${3:-577}
export TMPDIR=/tmp
mkdir -p "$OUT"
groups=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
  "SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU"
)
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc$i" -o run -- \
    python3 tools/attn_variants.py --eager 10 --seqs "$SEQ" --variants "$VAR" > "$OUT/pmc$i.log" 2>&1 \
    || { echo "pmc pass $i failed rc=$?"; tail -5 "$OUT/pmc$i.log"; exit 1; }
  i=$((i+1))
done
echo "pmc ok"
