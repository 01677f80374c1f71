#!/bin/bash
# Kernel trace of a short bench run; prints per-launch durations of the last chain.
# Usage (GPU box): bash tools/ktrace.sh <tag> <workload> [bench args ...]   (C2hot = C2 --params hot)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; wl=$2; shift 2
extra=""; [ "$wl" = "C2hot" ] && { wl=C2; extra="--params hot"; }
out=gpurun_out/kt_$tag
mkdir -p $out
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
  python3 bench.py --workload $wl $extra --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline "$@" > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
python3 tools/ktrace_summary.py $out
