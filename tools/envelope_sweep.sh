#!/bin/bash
# Envelope-solve tuning on the GPU box: C2 at P_FULL and P_HOT for each warm-up
# length given (super-tiles).  Usage: bash tools/envelope_sweep.sh 0 1 2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for w in "$@"; do
  for p in full hot; do
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --params $p --tune COMP_WARMUP=$w \
      > gpurun_out/env_${p}_w$w.json 2> gpurun_out/env_${p}_w$w.err || { tail -5 gpurun_out/env_${p}_w$w.err; exit 1; }
    python - "$p" "$w" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/env_{sys.argv[1]}_w{sys.argv[2]}.json").read().strip().splitlines()[-1])
c = d["chain"]; k = c["kernels_ms_per_step"]
print(f"{sys.argv[1]} W={sys.argv[2]}: {d['ms_per_step']:.4f} ms iters={c['comp_iters']} walked={c['comp_rewalked_frames']} "
      f"jumped={c.get('comp_jumped_frames')} pass0={k.get('comp_pass0')} fix={k.get('comp_fix')} refill={k.get('comp_refill')}", flush=True)
PY
  done
done
