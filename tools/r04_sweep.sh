#!/bin/bash
# Round-4 A/B sweep of bench tunes without the test suite: each argument is
# "tag:--tune A=1 --tune B=2" (bench arguments after the colon); every variant runs
# C2 and C2 P_HOT, and C3/C5 when SWEEP_ALL=1.  A tag var_<name> runs the ablation
# build build/var/<name>.so (tools/build_var.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --profile-steps 3 "$@" \
    > gpurun_out/sw_$tag.json 2> gpurun_out/sw_$tag.err || { echo "FAILED $tag"; tail -5 gpurun_out/sw_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sw_$tag.json')); k=d['chain']['kernels_ms_per_step']; print('$tag', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,2), 'G/s it', d['chain']['comp_iters'], 'rw', d['chain']['comp_rewalked_frames'], 'jmp', d['chain']['comp_jumped_frames'], {n: round(v,4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])[:11]})"
}
for v in "$@"; do
  tag=${v%%:*}; args=${v#*:}
  unset MM_LIB
  case $tag in var_*) export MM_LIB=$PWD/build/var/${tag#var_}.so ;; esac
  run ${tag}_C2 --workload C2 $args || exit 1
  run ${tag}_C2hot --workload C2 --params hot $args || exit 1
  if [ "$SWEEP_ALL" = 1 ]; then
    run ${tag}_C3 --workload C3 $args || exit 1
    run ${tag}_C5 --workload C5 $args || exit 1
  fi
done
