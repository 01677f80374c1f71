#!/bin/bash
# A/B: the round-3 start (git worktree in build/old, its own library) against this tree.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for side in old new; do
  dir=$GRAFT_REPO_ROOT; [ $side = old ] && dir=$GRAFT_REPO_ROOT/build/old
  for w in "C2 full" "C2 hot" "C3 full" "C5 full"; do
    set -- $w
    (cd $dir && timeout -k 10 200 python bench.py --workload $1 --params $2 --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 2) \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "$side $w failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/ab.json'));k=d['chain']['kernels_ms_per_step']
print('$side $w'.ljust(14), round(d['value']/1e9,3), round(d['ms_per_step'],3), 'it', d['chain']['comp_iters'], {n: round(v,4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])[:7]})"
  done
done
