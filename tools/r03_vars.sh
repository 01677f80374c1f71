#!/bin/bash
# Ablation builds (build/var/*.so) against the product library on P_FULL and P_HOT (C2 size).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "" $(ls build/var/*.so 2>/dev/null); do
  name=${lib:-base}; name=$(basename $name .so)
  for p in full hot; do
    MM_LIB=${lib:+$PWD/$lib} timeout -k 10 150 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --params $p --profile-steps 3 \
       > gpurun_out/var.json 2> gpurun_out/var.err || { echo "$name failed"; tail -5 gpurun_out/var.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/var.json'));k=d['chain']['kernels_ms_per_step']
print('$name $p'.ljust(16), round(d['ms_per_step'],3), 'it', d['chain']['comp_iters'], {n: round(v,4) for n, v in k.items() if n.startswith('comp')})"
  done
done
