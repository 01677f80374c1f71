#!/bin/bash
# gfx950 ISA of the library (hipcc --save-temps) for tools/isa_loops.py.
# Usage: bash tools/isa.sh <outdir> [extra hipcc flags...]   -> <outdir>/lib.s
src=$(cd "$(dirname "$0")/.." && pwd)/python-audio-mastering_amd/csrc/mastering.hip
out=${1:-/tmp/isa}; shift
mkdir -p $out && cd $out || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-value \
  -Wno-unused-result -DMM_SOURCE_SHA='"isa"' --save-temps "$@" -o $out/lib.so \
  $src -lrccl || exit 1
mv mastering-hip-amdgcn-amd-amdhsa-gfx950.s lib.s && rm -f mastering-*
