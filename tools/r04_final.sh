#!/bin/bash
# End-of-round measurement (round 4): GPU tests + smoke, then per workload the
# rocprofv3 kernel trace + PMC passes (summaries into profiles/r04_<w>_pmc_summary.json,
# copied to gpurun_out/profiles/) and the bench line that quotes them.
# Usage: bash tools/r04_final.sh [skip-tests] [workloads...]   (default: C2 C2hot C3 C4 C5 C1)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/profiles
if [ "$1" = "skip-tests" ]; then
  shift
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r04.log; [ $rc -ne 0 ] && exit $rc
fi
wls="$@"; [ -z "$wls" ] && wls="C2 C2hot C3 C4 C5 C1"
for w in $wls; do
  case $w in
    C2hot) wl=C2; args="--params hot" ;;
    *) wl=$w; args="" ;;
  esac
  if [ "$w" != C1 ]; then
    LABEL=r04_$w bash tools/pmc.sh r04$w $wl $args || exit 1
    cp profiles/r04_${w}_* gpurun_out/profiles/
  fi
  cb="--no-cpu-baseline"; case $w in C1|C2) cb="" ;; esac
  timeout -k 10 400 python -u bench.py --workload $wl $args $cb > gpurun_out/bench_r04_$w.json 2> gpurun_out/bench_r04_$w.err
  rc=$?; echo "bench $w rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r04_$w.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_r04_$w.json')); print('$w', round(d['value']/1e9,3), 'G frames/s', round(d['ms_per_step'],4), 'ms', 'traffic', d['roofline'].get('traffic'))"
done
