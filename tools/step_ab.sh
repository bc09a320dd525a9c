# whole C2 step (hipGraph) under alternative bench.py flag sets, interleaved rounds
# usage (GPU box): bash tools/step_ab.sh "--attn-variant 1" "--attn-variant 3" "--streams 3"
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in ${ROUNDS:-1 2}; do
  i=0
  for flags in "$@"; do
    timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-roofline --cpu-seconds 0 --no-modes --no-c5 \
      $flags > gpurun_out/sab_$i.json 2>/dev/null || exit 1
    echo "round $r [$flags] $(python -c "import json;d=json.load(open('gpurun_out/sab_$i.json'));print(d['value'], d['ms_per_step'])")"
    i=$((i+1))
  done
done
