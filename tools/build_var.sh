#!/bin/bash
# Ablation build of the library: bash tools/build_var.sh <name> -D<macro>=<value> ...
# -> build/abl/<name>.so (tools/ablate.sh times every build/abl/*.so against the product)
cd "$(dirname "$0")/../python-audio-mastering_amd" || exit 1
name=$1; shift
mkdir -p ../build/abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-value \
  -Wno-unused-result -DMM_SOURCE_SHA='"ablation"' "$@" -o ../build/abl/$name.so csrc/mastering.hip -lrccl 2>&1 | grep -E "error" 
exit 0
