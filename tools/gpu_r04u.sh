#!/bin/bash
# bf16 vs fp16 (contract mode): in-step one-stream per-op profile of each
set -o pipefail
mkdir -p gpurun_out/r04u
for dt in bf16 fp16; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-modes --no-c5 --dtype $dt \
    > gpurun_out/r04u/$dt.json 2>gpurun_out/r04u/$dt.err || exit 1
done
python - <<'PY'
import json
d = {dt: json.loads(open(f"gpurun_out/r04u/{dt}.json").readline()) for dt in ("bf16", "fp16")}
for dt in d:
    print(dt, d[dt]["value"], d[dt]["ms_per_step"])
a, b = (d[dt]["roofline"] for dt in ("bf16", "fp16"))
p = {dt: d[dt].get("step_profile", {}).get("one_stream", {}).get("by_op", {}) for dt in d}
for op in p["bf16"]:
    x, y = p["bf16"][op]["ms"], p["fp16"].get(op, {}).get("ms", 0)
    print(f"{op:14s} bf16 {x:7.3f} ms  fp16 {y:7.3f} ms  ratio {y / x if x else 0:5.3f}")
PY
