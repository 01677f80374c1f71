#!/bin/bash
# Warm-up length on the heavy-compression worst case (C2 at P_HOT thresholds) and P_FULL.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
# HOT_SPECS: space-separated params:warmup pairs
for spec in ${HOT_SPECS:-hot:6 hot:9 hot:12 hot:16 full:9}; do
  set -- ${spec/:/ }
  MM_COMP_WARMUP=$2 timeout -k 10 200 python -u bench.py --params $1 --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 2 > gpurun_out/hs.json 2> gpurun_out/hs.err
  rc=$?; [ $rc -ne 0 ] && { echo "$spec rc=$rc"; tail -5 gpurun_out/hs.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/hs.json')); k=d['chain']['kernels_ms_per_step']; print('$1 W=$2', round(d['ms_per_step'],3), 'ms it', d['chain']['comp_iters'], 'rw', d['chain']['comp_rewalked_frames'], 'pass0', k['comp_pass0'], 'fix', k['comp_fix'])"
done
