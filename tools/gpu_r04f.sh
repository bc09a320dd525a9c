# round-4: attention PMC, variant 3 (16x16, default) vs 6 (32x32 pipelined)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd $R
for v in 3 6; do
  bash tools/prof_pmc_attn.sh $R/gpurun_out/pmc_attn_v$v $v 577 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/pmc_attn_v3 --out gpurun_out/pmc_attn_v3/summary.json | grep attn
python3 tools/pmc_summary.py gpurun_out/pmc_attn_v6 --out gpurun_out/pmc_attn_v6/summary.json | grep attn
