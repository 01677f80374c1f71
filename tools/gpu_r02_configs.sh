#!/bin/bash
# Round-2 GPU run: the multi-track config tests (C3/C4/C5, P_HOT worst case) and
# the bench workloads.  Usage (GPU box): bash tools/gpu_r02_configs.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 1000 --timeout-method thread \
  > gpurun_out/configs_$tag.log 2>&1
rc=$?; tail -15 gpurun_out/configs_$tag.log; [ $rc -ne 0 ] && exit $rc
for w in C2 C3 C4 C5; do
  timeout -k 10 400 python -u bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 2 \
    > gpurun_out/bench_${tag}_$w.json 2> gpurun_out/bench_${tag}_$w.err
  rc=$?; echo "bench $w rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_${tag}_$w.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${tag}_$w.json')); print('$w', round(d['value']/1e9,3), 'Gfr/s', round(d['ms_per_step'],3), 'ms', d['roofline']['dominant_kernel']['name'])"
done
