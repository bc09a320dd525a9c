# C2 bench A/B over GEMM variants (interleaved, 2 rounds)
set -o pipefail
for r in 1 2; do
  for v in 0 4 3; do
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-modes --no-roofline --no-c5 --gemm-variant $v > gpurun_out/var_${v}_$r.json || exit 1
  done
done
