#!/bin/bash
# Build an A/B variant of libaaclip_hip.so with extra compile definitions, into ab/NAME.so
# (the build container; ab/ travels to the GPU box with the tree, tools/lib_ab.sh times it).
# usage: bash tools/ab_build.sh NAME -DAACLIP_WT_GEMM=1 [...]
set -e
NAME=$1
shift
R=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/aaclip_ab_build/$NAME
mkdir -p "$B" "$R/ab"
cd "$R/aa-clip_amd/csrc"
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics -I../../include"
for f in gemm attention rows anomaly_map metrics preprocess version; do
  extra=""
  [ $f = attention ] && extra=-fno-honor-nans
  /opt/rocm/bin/hipcc $FLAGS $extra "$@" -c $f.hip -o "$B/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o "$R/ab/$NAME.so" "$B"/*.o
echo "built ab/$NAME.so"
