# A/B of two builds of libaaclip_hip.so (AACLIP_LIB) on one box, interleaved rounds:
# the whole C2 step (bench.py, hipGraph) and, with ATTN=1, the attention kernel alone.
# usage (GPU box): [ROUNDS=3] bash tools/lib_ab.sh ab/libaaclip_base.so aa-clip_amd/aaclip/libaaclip_hip.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-3}); do
  for lib in "$@"; do
    if [ "${ATTN:-0}" = 1 ]; then
      AACLIP_LIB=$lib timeout -k 10 120 python tools/attn_variants.py --variants 3 --seqs 577,1025 \
        > gpurun_out/lab_attn.txt 2>&1 || exit 1
      echo "round $r $lib attn: $(grep -v amdgpu.ids gpurun_out/lab_attn.txt | tr '\n' ' ')"
    fi
    AACLIP_LIB=$lib timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-roofline --cpu-seconds 0 \
      --no-modes --no-c5 > gpurun_out/lab.json 2>/dev/null || exit 1
    echo "round $r $lib step: $(python -c "import json;d=json.load(open('gpurun_out/lab.json'));print(d['value'], d['ms_per_step'])")"
  done
done
