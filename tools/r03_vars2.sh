#!/bin/bash
# Ablation builds (build/var/*.so) against the product library: C2 P_FULL / P_HOT, C5;
# then C5 super-tile lengths on the first variant.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name lib workload params [tune]
  MM_LIB=$2 timeout -k 10 200 python bench.py --workload $3 --params $4 ${5:+--tune $5} --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 2 \
     > gpurun_out/var.json 2> gpurun_out/var.err || { echo "$1 failed"; tail -5 gpurun_out/var.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/var.json'));k=d['chain']['kernels_ms_per_step']
print('$1 $3 $4 $5'.ljust(34), round(d['value']/1e9,3), round(d['ms_per_step'],3), 'it', d['chain']['comp_iters'][:2], {n: round(v,4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])[:7]})"
}
for lib in "" $(ls build/var/*.so 2>/dev/null); do
  name=${lib:-base}; name=$(basename $name .so); l=${lib:+$PWD/$lib}
  run $name "$l" C2 full || exit 1
  run $name "$l" C2 hot || exit 1
  run $name "$l" C5 full || exit 1
done
v=$(ls build/var/*.so | head -1)
run tps16 $PWD/$v C5 full COMP_SUPER_FRAMES=918 || exit 1
run tps8 $PWD/$v C5 full COMP_SUPER_FRAMES=460 || exit 1
