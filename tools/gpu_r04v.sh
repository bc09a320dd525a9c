#!/bin/bash
# HIP runtime launch knobs in the C2 step: default vs HIP_FORCE_DEV_KERNARG=1 vs
# DEBUG_CLR_GRAPH_PACKET_CAPTURE=0/1 (interleaved rounds, same build)
set -o pipefail
mkdir -p gpurun_out/r04v
for r in 1 2 3; do
  for env in "X=0" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
    env $env timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-roofline --cpu-seconds 0 --no-modes --no-c5 \
      > gpurun_out/r04v/b.json 2>/dev/null || exit 1
    echo "round $r $env $(python -c "import json;d=json.load(open('gpurun_out/r04v/b.json'));print(d['value'], d['ms_per_step'])")"
  done
done | tee gpurun_out/r04v/ab.txt
