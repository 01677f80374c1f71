#!/bin/bash
# Development round trip on the GPU box: GPU tests (stop at the first failure),
# then bench lines of the given workloads (default C2 C2hot).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_chk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_chk.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_all.sh chk ${@:-C2 C2hot}
