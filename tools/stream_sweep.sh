# C2 + C5 throughput vs concurrent image chunks (HIP streams) per GPU
set -o pipefail
for s in 1 2 3 4; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-modes --no-roofline --streams $s > gpurun_out/streams_$s.json || exit 1
done
