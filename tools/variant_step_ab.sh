# whole C2 step (two streams, hipGraph) under GEMM tile-family overrides, interleaved rounds
# usage (GPU box): bash tools/variant_step_ab.sh "0 3 5" ["--streams 1"]
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in $1; do
    timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-roofline --cpu-seconds 0 --no-modes --no-c5 \
      --gemm-variant $v $2 > gpurun_out/vab_$v.json 2>/dev/null || exit 1
    echo "round $r variant $v $(python -c "import json;d=json.load(open('gpurun_out/vab_$v.json'));print(d['value'], d['ms_per_step'])")"
  done
done
