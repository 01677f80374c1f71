#!/bin/bash
# pass0 warm-up sweep: exact warm-up W and coarse warm-up C (super-tiles).
# Usage (GPU box): bash tools/warm_sweep.sh ["W:C W:C ..."]
cd $GRAFT_REPO_ROOT
for wc in ${1:-6:0 4:0}; do
  w=${wc%:*}; c=${wc#*:}
  MM_COMP_WARMUP=$w MM_COMP_WARM_COARSE=$c timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --profile-steps 3 > gpurun_out/warm_${w}_${c}.json 2>/dev/null || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/warm_${w}_${c}.json'));c=d['chain'];k=c['kernels_ms_per_step'];print('W=$w C=$c', round(d['ms_per_step'],3), 'iters',c['comp_iters'],'walked',c['comp_rewalked_frames'],'pass0',k['comp_pass0'],'fix',k['comp_fix'],'record',k.get('comp_record'))"
done
