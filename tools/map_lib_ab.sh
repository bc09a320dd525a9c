# A/B of the anomaly map inside the C2 step: the in-step figure (bench.py's
# roofline_map, HIP events around the op) and the whole step, interleaved rounds so
# clock drift hits every arm alike. Arms: "lib:fused" = AACLIP_LIB=lib with
# AACLIP_MAP_FUSED=fused (1 = one-launch aaclip_anomaly_map_fused, 0 = two launches).
# usage (GPU box): bash tools/map_lib_ab.sh ab/libaaclip_base.so:0 aa-clip_amd/aaclip/libaaclip_hip.so:0 \
#                  aa-clip_amd/aaclip/libaaclip_hip.so:1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do
  for arm in "$@"; do
    lib=${arm%%:*}; fused=${arm##*:}
    AACLIP_LIB=$lib AACLIP_MAP_FUSED=$fused timeout -k 10 180 python bench.py --steps 20 --warmup 3 \
      --cpu-seconds 0 --no-modes --no-c5 > gpurun_out/mab.json 2>/dev/null || exit 1
    echo "round $r $arm: $(python -c "
import json;d=json.load(open('gpurun_out/mab.json'));m=d.get('roofline_map',{})
print('step', d['value'], d['ms_per_step'], 'map_us', m.get('avg_launch_us'), 'frac', m.get('frac'),
      '2stream_us', m.get('in_step_2stream',{}).get('avg_launch_us'))")"
  done
done
