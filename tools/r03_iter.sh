#!/bin/bash
# Development round trip: GPU tests, sweep traces, ablation builds, bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_chk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_chk.log
[ $rc -eq 0 ] || exit $rc
bash tools/fix_trace.sh C2 && bash tools/fix_trace.sh C2hot || exit 1
bash tools/ablate.sh comp_pass0 comp_fix comp_rms comp_apply || exit 1
bash tools/gpu_bench_all.sh chk ${@:-C2 C2hot C3 C5}
