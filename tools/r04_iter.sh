#!/bin/bash
# Round-4 development round trip: GPU tests, then bench lines of C2 / C2hot, A/B
# variants (environment settings "ENV=x" or bench tunes "tune:NAME=V"), sweep-walker
# cost fits, C3 / C5.
# Usage: bash tools/r04_iter.sh [skip-tests] [variants...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$1" = "skip-tests" ]; then
  shift
else
  timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_iter.log
  [ $rc -eq 0 ] || exit $rc
fi
run() {  # tag, env (or -), bench args
  local tag=$1 envs=$2; shift 2
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --profile-steps 3 "$@" \
    > gpurun_out/it_$tag.json 2> gpurun_out/it_$tag.err || { echo "FAILED $tag"; tail -5 gpurun_out/it_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/it_$tag.json')); k=d['chain']['kernels_ms_per_step']; print('$tag', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,2), 'G/s it', d['chain']['comp_iters'], 'rw', d['chain']['comp_rewalked_frames'], 'jmp', d['chain']['comp_jumped_frames'], {n: round(v,4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])[:11]})"
}
run C2 - --workload C2 || exit 1
run C2hot - --workload C2 --params hot || exit 1
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "${v#tune:}" != "$v" ]; then
    run C2_v$i - --workload C2 --tune ${v#tune:} || exit 1
    run C2hot_v$i - --workload C2 --params hot --tune ${v#tune:} || exit 1
  else
    run C2_v$i "$v" --workload C2 || exit 1
    run C2hot_v$i "$v" --workload C2 --params hot || exit 1
  fi
  echo "  (v$i = $v)"
done
for w in C2 C2hot; do
  extra=""; [ "$w" = "C2hot" ] && extra="--params hot"
  MM_FIX_TRACE=1 MM_FIX_TRACE_DUMP=gpurun_out/fixdump_$w.bin timeout -k 10 200 python -u bench.py --workload C2 $extra \
    --steps 1 --warmup 1 --profile-steps 1 --no-cpu-baseline > gpurun_out/ft_$w.json 2> gpurun_out/ft_$w.err \
    || { tail -5 gpurun_out/ft_$w.err; exit 1; }
  echo "fix trace $w"; python tools/fix_fit.py gpurun_out/fixdump_$w.bin
done
for lib in $(ls build/var/*.so 2>/dev/null); do
  run C2_$(basename $lib .so) "MM_LIB=$PWD/$lib" --workload C2 || exit 1
done
run C3 - --workload C3 || exit 1
run C5 - --workload C5 || exit 1
