#!/bin/bash
# Development GPU round trip: parity + full-size tests, then the C2/C3/C5 benches.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py ${FZ_TESTS} -x -v --timeout 300 --timeout-method thread > gpurun_out/fz_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/fz_test.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/fz_test.log | head -20; exit $rc; }
for w in ${FZ_WL:-C2 C3 C5}; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 2 > gpurun_out/fz_bench_$w.json 2> gpurun_out/fz_bench_$w.err
  rc=$?; echo "bench $w rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/fz_bench_$w.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/fz_bench_$w.json')); print('$w', round(d['value']/1e9,3), 'Gfr/s', round(d['ms_per_step'],3), 'ms', d['chain']['kernels_ms_per_step'])"
done
