#!/bin/bash
# envelope solve shape sweep: warm-up W (super-tiles) x super-tile size U (active frames).
# Usage (GPU box): bash tools/super_sweep.sh ["W:U W:U ..."]
cd $GRAFT_REPO_ROOT
for wu in ${1:-6:1000 6:500}; do
  w=${wu%:*}; u=${wu#*:}
  MM_COMP_WARMUP=$w MM_COMP_SUPER=$u timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --profile-steps 3 > gpurun_out/sw_${w}_${u}.json 2>/dev/null || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/sw_${w}_${u}.json'));c=d['chain'];k=c['kernels_ms_per_step'];print('W=$w U=$u', round(d['ms_per_step'],3), 'iters',c['comp_iters'],'walked',c['comp_rewalked_frames'],'pass0',k['comp_pass0'],'fix',k['comp_fix'],'record',k.get('comp_record'),'compact',k['comp_compact'])"
done
