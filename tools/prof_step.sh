# rocprofv3 kernel trace of the bare C2 step (bench.py, no extra legs), one and two streams.
# usage (GPU box): bash tools/prof_step.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/step_prof}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
for s in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/s$s -o run -- python3 $R/bench.py --steps 5 --warmup 2 \
    --streams $s --no-roofline --cpu-seconds 0 --no-modes --no-c5 > $R/$OUT/s$s.log 2>&1 || exit $?
  python3 $R/tools/trace_summary.py $(find $R/$OUT/s$s -name "*kernel_trace.csv" | head -1) --out $R/$OUT/s$s.json --timeline > $R/$OUT/s$s.txt || exit $?
done
