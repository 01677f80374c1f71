#!/bin/bash
# Probes: pass 0 without describers, ablation builds, warm-up 1, super-tile sizes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/env_sweep.sh probe C2 "MM_COMP_NOJUMP=1" "MM_X=0" || exit 1
bash tools/ablate.sh comp_pass0 comp_fix comp_rms comp_apply || exit 1
for t in "COMP_WARMUP=1" "COMP_SUPER_FRAMES=500" "COMP_SUPER_FRAMES=750" "COMP_SUPER_FRAMES=1500"; do
  for p in full hot; do
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --params $p --tune $t --profile-steps 2 \
      > gpurun_out/tune.json 2> gpurun_out/tune.err || { tail -5 gpurun_out/tune.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/tune.json'));k=d['chain']['kernels_ms_per_step']
print('$t $p', round(d['ms_per_step'],3), 'it', d['chain']['comp_iters'], {n: round(v,4) for n, v in k.items() if n.startswith('comp')})"
  done
done
