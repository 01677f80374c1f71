#!/bin/bash
# Per-kernel device times of ablation builds (build/var/*.so, made with -D<macro>)
# against the product library.  Usage (GPU box): bash tools/ablate.sh [kernel ...]
cd "$GRAFT_REPO_ROOT" || exit 1
ks=${*:-eq xover}
for lib in "" $(ls build/var/*.so 2>/dev/null); do
  name=${lib:-base}
  MM_LIB=${lib:+$PWD/$lib} timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 3 \
     > gpurun_out/abl.json 2> gpurun_out/abl.err || { echo "$name failed"; tail -5 gpurun_out/abl.err; exit 1; }
  python -c "
import json,sys;d=json.load(open('gpurun_out/abl.json'));k=d['chain']['kernels_ms_per_step']
print('$name'.ljust(28), round(d['ms_per_step'],3), 'it', d['chain']['comp_iters'], 'rw', d['chain']['comp_rewalked_frames'], ' '.join(f'{x}={k.get(x)}' for x in '$ks'.split()))"
done
