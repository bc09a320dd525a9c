set -o pipefail
# marginal step cost per op: apply tools/diag_skip.patch first (git apply), run on the GPU box, revert after
# (the skipped ops leave stale but realistic activations; outputs are wrong by construction)
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  i=0
  for v in none attn qkv out fc proj ln2,tail attn,ln2,tail; do
    AACLIP_DIAG_SKIP=$v timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-roofline --cpu-seconds 0 --no-modes --no-c5 > gpurun_out/diag_$i.json 2>gpurun_out/diag_$i.err || exit 1
    echo "round $r skip=$v $(python -c "import json;d=json.load(open('gpurun_out/diag_$i.json'));print(d['value'], d['ms_per_step'])")"
    i=$((i+1))
  done
done
