#!/bin/bash
# One GPU-box recipe for A/B and measurement runs (replaces the round-4 one-off
# gpu_r04*.sh scripts; their command lines are in the git history before round 5):
# every argument is one command, run from the repo root under its own time limit, its
# output kept in gpurun_out/TAG/NN.log; the recipe stops at the first failing command
# (fault, abort, time limit) so nothing else touches a GPU in a bad state.
# usage (GPU box): [LIMIT=300] bash tools/gpu_ab.sh TAG 'cmd 1' 'cmd 2' ...
# e.g.  bash tools/gpu_ab.sh r05x 'bash tools/lib_ab.sh ab/base.so aa-clip_amd/aaclip/libaaclip_hip.so' \
#          'python tools/attn_variants.py --variants 1,3 --seqs 577,1025'
set -o pipefail
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
i=0
for cmd in "$@"; do
  i=$((i + 1))
  log=$OUT/$(printf %02d $i).log
  echo "# $cmd" > "$log"
  timeout -k 10 "${LIMIT:-300}" bash -c "$cmd" >> "$log" 2>&1
  rc=$?
  echo "[$i] rc=$rc: $cmd"
  tail -"${TAIL:-6}" "$log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
