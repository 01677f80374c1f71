#!/bin/bash
# Bench lines of several library builds on several workloads, on one box:
#   bash tools/ab_lines.sh "C2 C3" - build/ab/x.so ...    ("-" = the in-tree library)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
wls=$1; shift
for v in "$@"; do
  for w in $wls; do
    if [ "$v" = "-" ]; then lib=""; tag=product; else lib=$PWD/$v; tag=$(basename "$v" .so); fi
    MM_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --profile-steps 3 \
      --workload $w > gpurun_out/ab_${w}_$tag.json 2> gpurun_out/ab_${w}_$tag.err || { echo "FAILED $w $tag"; tail -5 gpurun_out/ab_${w}_$tag.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${w}_$tag.json')); k=d['chain']['kernels_ms_per_step']; print('$w', '$tag', round(d['ms_per_step'],4), 'ms', {n: round(x,4) for n, x in sorted(k.items(), key=lambda kv: -kv[1])[:6]})"
  done
done
