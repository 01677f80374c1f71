#!/bin/bash
# Round-4 development round trip: GPU tests, then bench lines of C2 / C2hot / C3 / C5
# (with optional --tune variants), per-kernel times.
# Usage: bash tools/r04_iter.sh [skip-tests] [tune settings...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$1" = "skip-tests" ]; then
  shift
else
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_iter.log
  [ $rc -eq 0 ] || exit $rc
fi
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --profile-steps 3 "$@" \
    > gpurun_out/it_$tag.json 2> gpurun_out/it_$tag.err || { echo "FAILED $tag"; tail -5 gpurun_out/it_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/it_$tag.json')); k=d['chain']['kernels_ms_per_step']; print('$tag', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,2), 'G/s it', d['chain']['comp_iters'], 'rw', d['chain']['comp_rewalked_frames'], {n: round(v,4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])[:10]})"
}
run C2 --workload C2 || exit 1
run C2hot --workload C2 --params hot || exit 1
for t in "$@"; do
  run C2_$t --workload C2 --tune $t || exit 1
  run C2hot_$t --workload C2 --params hot --tune $t || exit 1
done
run C3 --workload C3 || exit 1
run C5 --workload C5 || exit 1
