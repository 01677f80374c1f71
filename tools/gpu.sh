#!/bin/bash
# The one GPU-box driver (replaces the per-round r0x_*.sh scripts).  Every step
# runs under its own time limit; the first failure ends the call.
#
#   bash tools/gpu.sh test [pytest selection...]      GPU parity suite (+ smoke)
#   bash tools/gpu.sh iter [variants...]              C2 / C2 P_HOT bench lines with the
#        per-kernel split; a variant is "ENV=x" (library env knob), "tune:NAME=V"
#        (bench tune) or "lib:<path.so>" (an ablation build from tools/build_var.sh)
#   bash tools/gpu.sh c2 [variants...]                C2 lines only (variants as in iter)
#   bash tools/gpu.sh configs [C3 C4 C5 C1 ...]       bench lines of the other workloads
#   bash tools/gpu.sh measure <round> [notest] [workloads...]  end-of-round measurement: tests, smoke,
#        per workload the rocprofv3 trace + PMC passes (tools/pmc.sh ->
#        profiles/<round>_<w>_pmc_summary.json) and the bench line quoting them
#   bash tools/gpu.sh lines <round> [workloads...]    the bench lines alone, quoting profiles/ as they are
#   bash tools/gpu.sh firstcall                       first master_pcm on a fresh context
#
# Several modes may be chained in one call: bash tools/gpu.sh test -- iter -- configs C3
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out gpurun_out/profiles

bench_line() {  # tag, env-or-"-", bench args...
  local tag=$1 envs=$2; shift 2
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --profile-steps 3 "$@" \
    > gpurun_out/it_$tag.json 2> gpurun_out/it_$tag.err || { echo "FAILED $tag"; tail -5 gpurun_out/it_$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/it_$tag.json')); k=d['chain']['kernels_ms_per_step']; print('$tag', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,2), 'G/s it', d['chain']['comp_iters'], {n: round(v,4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])[:12]})"
}

mode_test() {
  timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  local rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || return $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; return $rc
}

mode_iter() {
  bench_line C2 - --workload C2 || return 1
  bench_line C2hot - --workload C2 --params hot || return 1
  local i=0 v
  for v in "$@"; do
    i=$((i + 1))
    case $v in
      tune:*) bench_line C2_v$i - --workload C2 --tune ${v#tune:} && \
              bench_line C2hot_v$i - --workload C2 --params hot --tune ${v#tune:} || return 1 ;;
      lib:*)  bench_line C2_v$i "MM_LIB=$PWD/${v#lib:}" --workload C2 && \
              bench_line C2hot_v$i "MM_LIB=$PWD/${v#lib:}" --workload C2 --params hot || return 1 ;;
      *)      bench_line C2_v$i "$v" --workload C2 && bench_line C2hot_v$i "$v" --workload C2 --params hot || return 1 ;;
    esac
    echo "  (v$i = $v)"
  done
}

mode_c2() {  # C2 lines only (P_FULL): the product, then each variant (as in iter)
  bench_line C2 - --workload C2 || return 1
  local i=0 v
  for v in "$@"; do
    i=$((i + 1))
    case $v in
      tune:*) bench_line C2_v$i - --workload C2 --tune ${v#tune:} || return 1 ;;
      lib:*)  bench_line C2_v$i "MM_LIB=$PWD/${v#lib:}" --workload C2 || return 1 ;;
      *)      bench_line C2_v$i "$v" --workload C2 || return 1 ;;
    esac
    echo "  (v$i = $v)"
  done
}

mode_configs() {
  local w
  for w in ${@:-C3 C5}; do bench_line $w - --workload $w || return 1; done
}

mode_measure() {  # measure <round> [notest] [workloads...]
  local round=$1; shift
  local skip_test=0; [ "$1" = "notest" ] && { skip_test=1; shift; }
  local wls="$@"; [ -z "$wls" ] && wls="C2 C2hot C3 C4 C5 C1"
  [ $skip_test -eq 1 ] || mode_test || return 1
  local w wl args cb
  for w in $wls; do
    case $w in C2hot) wl=C2; args="--params hot" ;; *) wl=$w; args="" ;; esac
    LABEL=${round}_$w bash tools/pmc.sh ${round}$w $wl $args || return 1
    cp profiles/${round}_${w}_* gpurun_out/profiles/
    cb="--no-cpu-baseline"; case $w in C1|C2) cb="" ;; esac
    timeout -k 10 400 python -u bench.py --workload $wl $args $cb > gpurun_out/bench_${round}_$w.json \
      2> gpurun_out/bench_${round}_$w.err
    local rc=$?; echo "bench $w rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_${round}_$w.err; return $rc; }
    python -c "import json; d=json.load(open('gpurun_out/bench_${round}_$w.json')); print('$w', round(d['value']/1e9,3), 'G frames/s', round(d['ms_per_step'],4), 'ms', 'traffic', d['roofline'].get('traffic'))"
  done
}

mode_lines() {  # lines <round> [workloads...]: the bench lines alone (profiles already in profiles/)
  local round=$1; shift
  local w wl args cb
  for w in ${@:-C2 C2hot C3 C4 C5 C1}; do
    case $w in C2hot) wl=C2; args="--params hot" ;; *) wl=$w; args="" ;; esac
    cb="--no-cpu-baseline"; case $w in C1|C2) cb="" ;; esac
    timeout -k 10 400 python -u bench.py --workload $wl $args $cb > gpurun_out/bench_${round}_$w.json \
      2> gpurun_out/bench_${round}_$w.err
    local rc=$?; echo "bench $w rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_${round}_$w.err; return $rc; }
    python -c "import json; d=json.load(open('gpurun_out/bench_${round}_$w.json')); print('$w', round(d['value']/1e9,3), 'G frames/s', round(d['ms_per_step'],4), 'ms', 'traffic', d['roofline'].get('traffic'))"
  done
}

mode_firstcall() {
  timeout -k 10 300 python -u tools/first_call.py > gpurun_out/first_call.json 2> gpurun_out/first_call.err
  local rc=$?; echo "first_call rc=$rc"; cat gpurun_out/first_call.json; [ $rc -eq 0 ] || tail -5 gpurun_out/first_call.err
  return $rc
}

# split the arguments at "--" into mode invocations
args=("$@")
start=0
for ((i = 0; i <= ${#args[@]}; i++)); do
  if [ $i -eq ${#args[@]} ] || [ "${args[$i]}" = "--" ]; then
    seg=("${args[@]:$start:$((i - start))}")
    start=$((i + 1))
    [ ${#seg[@]} -eq 0 ] && continue
    m=${seg[0]}
    mode_$m "${seg[@]:1}" || exit 1
  fi
done
