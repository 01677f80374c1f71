#!/bin/bash
# Probes of the envelope-solve geometry: sweep-walker traces, then warm-up and
# super-tile length (engine knobs) on P_FULL and P_HOT at C2 size.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/fix_trace.sh C2 && bash tools/fix_trace.sh C2hot || exit 1
for t in "COMP_WARMUP=0" "COMP_WARMUP=1" "COMP_SUPER_FRAMES=500" "COMP_SUPER_FRAMES=750" "COMP_SUPER_FRAMES=1500" "COMP_SUPER_FRAMES=2000"; do
  for p in full hot; do
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --params $p --tune $t --profile-steps 2 \
      > gpurun_out/tune.json 2> gpurun_out/tune.err || { tail -5 gpurun_out/tune.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/tune.json'));k=d['chain']['kernels_ms_per_step']
print('$t $p', round(d['ms_per_step'],3), 'it', d['chain']['comp_iters'], 'rw', d['chain']['comp_rewalked_frames'], 'jp', d['chain']['comp_jumped_frames'], {n: round(v,4) for n, v in k.items() if n.startswith('comp')})"
  done
done
