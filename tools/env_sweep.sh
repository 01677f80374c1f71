#!/bin/bash
# Bench one workload under several environment settings (tuning knobs such as
# MM_COMP_LAYOUT, MM_PASS0_OWN), printing step time and the top kernels.
# Usage: bash tools/env_sweep.sh <tag> <workload|C2hot> "ENV=a ENV2=b" "ENV=c" ...
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; w=$2; shift 2
mkdir -p gpurun_out
extra=""; wl=$w
[ "$w" = "C2hot" ] && { wl=C2; extra="--params hot"; }
i=0
for setting in "$@"; do
  i=$((i+1))
  out=gpurun_out/sweep_${tag}_${w}_$i
  env $setting timeout -k 10 300 python -u bench.py --workload $wl $extra --no-cpu-baseline --steps 10 --warmup 3 --profile-steps 3 \
    > $out.json 2> $out.err || { echo "FAILED: $setting"; tail -5 $out.err; exit 1; }
  python -c "import json; d=json.load(open('$out.json')); k=d['chain']['kernels_ms_per_step']; print('$w [$setting]', round(d['ms_per_step'],4), 'ms', 'iters', d['chain']['comp_iters'], 'walked', d['chain']['comp_rewalked_frames'], {n: round(v,4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])[:9]})"
done
