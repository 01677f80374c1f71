#!/bin/bash
# pass-0 ownership sweep (MM_PASS0_OWN) on C2 and C4: bash tools/own_sweep.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-own}
mkdir -p gpurun_out
for w in C2 C4; do for o in 1 2 4 8; do
  MM_PASS0_OWN=$o timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 2 \
    > gpurun_out/own_${tag}_${w}_$o.json 2> gpurun_out/own_${tag}_${w}_$o.err || { tail -5 gpurun_out/own_${tag}_${w}_$o.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/own_${tag}_${w}_$o.json')); k=d['chain']['kernels_ms_per_step']; print('$w own=$o', round(d['ms_per_step'],3), 'ms pass0', k['comp_pass0'], 'fix', k.get('comp_fix'), 'iters', d['chain']['comp_iters'])"
done; done
