cd "$GRAFT_REPO_ROOT" || exit 1
for spec in 1000:6:0 500:12:0 500:12:4 500:10:2 750:8:0; do
  set -- ${spec//:/ }
  MM_COMP_SUPER=$1 MM_COMP_WARMUP=$2 MM_PASS0_OWN=$3 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 --profile-steps 1 > gpurun_out/u.json 2> gpurun_out/u.err || { tail -3 gpurun_out/u.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/u.json')); k=d['chain']['kernels_ms_per_step']; print('U=$1 W=$2 own=$3', round(d['ms_per_step'],3), 'ms', {x: k[x] for x in ('comp_compact','comp_pass0','comp_fix','comp_apply')}, d['chain']['comp_rewalked_frames'])"
done
