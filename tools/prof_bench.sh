# rocprofv3 kernel trace + stats of the default bench.py command (the line the driver
# runs), and the per-(kernel, grid) summary that checks the line's in-step figures.
# usage (GPU box): bash tools/prof_bench.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/prof_bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $R/bench.py \
  > $R/$OUT/bench.json 2> $R/$OUT/bench.err || exit $?
python3 $R/tools/trace_summary.py $(find $R/$OUT/trace -name "*kernel_trace.csv" | head -1) --out $R/$OUT/per_grid.json \
  > $R/$OUT/per_grid.txt || exit $?
cp $(find $R/$OUT/trace -name "*kernel_stats.csv" | head -1) $R/$OUT/kernel_stats.csv
