cd $GRAFT_REPO_ROOT
for w in 5 6 7; do MM_COMP_WARMUP=$w timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --profile-steps 3 > gpurun_out/warm_$w.json 2>/dev/null || exit 1; python -c "
import json;d=json.load(open('gpurun_out/warm_$w.json'));c=d['chain'];k=c['kernels_ms_per_step'];print('W=$w', round(d['ms_per_step'],3), 'iters',c['comp_iters'],'walked',c['comp_rewalked_frames'],'pass0',k['comp_pass0'],'fix',k['comp_fix'],'record',k['comp_record'])"; done
