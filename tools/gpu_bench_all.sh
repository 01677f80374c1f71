#!/bin/bash
# Bench every workload (C2..C5, plus C2 with P_HOT) on the GPU box, no CPU leg.
# Usage: bash tools/gpu_bench_all.sh <tag> [workloads...]
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r02}; shift
ws=${@:-C2 C2hot C3 C4 C5}
mkdir -p gpurun_out
for w in $ws; do
  extra=""; wl=$w
  [ "$w" = "C2hot" ] && { wl=C2; extra="--params hot"; }
  timeout -k 10 400 python -u bench.py --workload $wl $extra --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 2 \
    > gpurun_out/bench_${tag}_$w.json 2> gpurun_out/bench_${tag}_$w.err
  rc=$?; echo "bench $w rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_${tag}_$w.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${tag}_$w.json')); print('$w', round(d['value']/1e9,3), 'Gfr/s', round(d['ms_per_step'],3), 'ms/step', d['roofline']['dominant_kernel']['name'], d['chain']['comp_iters'], {k: v for k, v in sorted(d['chain']['kernels_ms_per_step'].items(), key=lambda kv: -kv[1])[:6]})"
done
