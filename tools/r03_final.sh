#!/bin/bash
# End-of-round measurement: GPU tests, rocprofv3 trace + PMC passes of C2 (the
# summary lands in profiles/ so the bench lines below carry `traffic`), then the
# bench line of every workload (C2 and C1 with the CPU baseline).
# Usage: bash tools/r03_final.sh [skip-tests]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/profiles
if [ "$1" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r03.log; [ $rc -ne 0 ] && exit $rc
fi
bash tools/pmc.sh r03 C2 || exit 1
cp profiles/r03_C2_* gpurun_out/profiles/
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r03_C2.json 2> gpurun_out/bench_r03_C2.err
rc=$?; echo "bench C2 rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r03_C2.err; exit $rc; }
for spec in "C1 --workload C1" "C2hot --workload C2 --params hot --no-cpu-baseline" "C3 --workload C3 --no-cpu-baseline" \
            "C4 --workload C4 --no-cpu-baseline" "C5 --workload C5 --no-cpu-baseline"; do
  set -- $spec; tag=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench_r03_$tag.json 2> gpurun_out/bench_r03_$tag.err
  rc=$?; echo "bench $tag rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r03_$tag.err; exit $rc; }
done
for f in gpurun_out/bench_r03_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e9,3), 'Gfr/s', round(d['ms_per_step'],3), 'ms')"; done
