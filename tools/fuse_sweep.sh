#!/bin/bash
# Unit-size sweep of the fused batch path: bench.py C3/C5 at several MM_FUSE_MAX_FRAMES.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in ${FUSE_SPECS:-"C5 0" "C5 35000000" "C5 140000000" "C5 300000000" "C3 16000000" "C3 32000000"}; do
  set -- $spec
  MM_FUSE_MAX_FRAMES=$2 timeout -k 10 300 python -u bench.py --workload $1 --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 1 > gpurun_out/fs.json 2> gpurun_out/fs.err
  rc=$?; [ $rc -ne 0 ] && { echo "$spec rc=$rc"; tail -5 gpurun_out/fs.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/fs.json')); print('$1 cap=$2', round(d['value']/1e9,3), 'Gfr/s', round(d['ms_per_step'],3), 'ms')"
done
