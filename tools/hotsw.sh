#!/bin/bash
# C2 at P_HOT with N queued fix sweeps: bash tools/hotsw.sh 4 6 8
cd "$GRAFT_REPO_ROOT" || exit 1
for n in "$@"; do
  MM_COMP_SWEEPS=$n timeout -k 10 120 python bench.py --params hot --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 3 \
     > gpurun_out/hs.json 2> gpurun_out/hs.err || { tail -5 gpurun_out/hs.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/hs.json'));c=d['chain'];k=c['kernels_ms_per_step']
print('sweeps $n', round(d['ms_per_step'],3), 'it', c['comp_iters'], 'rw', c['comp_rewalked_frames'], k)"
done
