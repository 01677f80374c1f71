#!/bin/bash
# Ablation build of the library: bash tools/build_var.sh <name> -D<macro>=<value> ...
# -> build/ab/<name>.so (travels to the GPU box: delete after the A/B; build/abl is gpurun-ignored)
cd "$(dirname "$0")/../python-audio-mastering_amd" || exit 1
name=$1; shift
mkdir -p ../build/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-value \
  -Wno-unused-result -DMM_SOURCE_SHA='"ablation"' "$@" -o ../build/ab/$name.so csrc/mastering.hip -lrccl 2>&1 | grep -E "error" 
exit 0
