#!/bin/bash
# Round-3 baseline on the GPU box: GPU tests, bench lines, envelope warm-up sweep.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_r03a.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_bench_all.sh r03a C2 C2hot C3 C5 || exit 1
bash tools/envelope_sweep.sh 0 2 6
