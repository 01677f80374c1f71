#!/bin/bash
# Tile length (MM_TILE) and super-tile length (MM_COMP_SUPER, 0 = default) on C2 / C3:
# TILE_SPECS = workload:tile:super triples.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in ${TILE_SPECS:-C2:125 C2:105 C2:147 C2:175 C3:125 C3:175}; do
  set -- ${spec//:/ }
  sup=${3:-1000}
  MM_TILE=$2 MM_COMP_SUPER=$sup timeout -k 10 300 python -u bench.py --workload $1 ${4:+--params $4} --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 1 > gpurun_out/ts.json 2> gpurun_out/ts.err
  rc=$?; [ $rc -ne 0 ] && { echo "$spec rc=$rc"; tail -5 gpurun_out/ts.err; continue; }
  python -c "import json; d=json.load(open('gpurun_out/ts.json')); k=d['chain']['kernels_ms_per_step']; print('$1 T=$2 U=$3', round(d['ms_per_step'],3), 'ms', {x: k[x] for x in ('eq','xover','comp_rms','comp_compact','comp_pass0','comp_apply','kweight')})"
done
