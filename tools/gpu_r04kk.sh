#!/bin/bash
# final tree: the default bench line twice on one fresh box (box-level spread of the headline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04kk
for r in 1 2; do
  timeout -k 10 600 python -u bench.py > gpurun_out/r04kk/bench_$r.json 2> gpurun_out/r04kk/bench_$r.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r04kk/bench_$r.json'));print($r, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['attn_mlp_block']['tflops'])"
done
