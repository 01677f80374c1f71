#!/bin/bash
# Pass-0 ownership on the batched workloads: OWN_SPECS = workload:own pairs (own 0 = host default).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in ${OWN_SPECS:-C3:0 C3:6 C3:8 C5:0 C5:8}; do
  set -- ${spec/:/ }
  MM_PASS0_OWN=$2 timeout -k 10 300 python -u bench.py --workload $1 --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 1 > gpurun_out/os.json 2> gpurun_out/os.err
  rc=$?; [ $rc -ne 0 ] && { echo "$spec rc=$rc"; tail -5 gpurun_out/os.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/os.json')); k=d['chain']['kernels_ms_per_step']; print('$1 own=$2', round(d['value']/1e9,3), 'Gfr/s', round(d['ms_per_step'],3), 'ms pass0', k['comp_pass0'], 'fix', k['comp_fix'], 'rw', d['chain']['comp_rewalked_frames'])"
done
