#!/bin/bash
# End-of-round measurement, part A: GPU tests, then the bench lines of every
# workload (C2 with the CPU baseline).  Part B is tools/pmc.sh r02 C2.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_r02.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r02.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r02_C2.json 2> gpurun_out/bench_r02_C2.err
rc=$?; echo "bench C2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r02_C2.err; exit $rc; }
for spec in "C2hot --workload C2 --params hot" "C3 --workload C3" "C4 --workload C4" "C5 --workload C5"; do
  set -- $spec; tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_r02_$tag.json 2> gpurun_out/bench_r02_$tag.err
  rc=$?; echo "bench $tag rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r02_$tag.err; exit $rc; }
done
for f in gpurun_out/bench_r02_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e9,3), 'Gfr/s', round(d['ms_per_step'],3), 'ms')"; done
