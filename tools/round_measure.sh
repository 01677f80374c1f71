#!/bin/bash
# Full measurement round on the GPU box: parity tests, bench (with CPU baseline),
# rocprofv3 trace + PMC passes.  Usage: bash tools/round_measure.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$tag.err; exit $rc; }
bash tools/pmc.sh $tag
