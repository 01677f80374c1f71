#!/bin/bash
# Sweep-walker trace (MM_FIX_TRACE): the slowest walkers of every fix-up sweep.
# Usage (GPU box): bash tools/fix_trace.sh <workload|C2hot> [env settings...]
cd "$GRAFT_REPO_ROOT" || exit 1
w=$1; shift
extra=""; wl=$w
[ "$w" = "C2hot" ] && { wl=C2; extra="--params hot"; }
env MM_FIX_TRACE=1 "$@" timeout -k 10 200 python -u bench.py --workload $wl $extra --steps 1 --warmup 1 --profile-steps 1 --no-cpu-baseline \
  > gpurun_out/ft_$w.json 2> gpurun_out/ft_$w.err || { tail -5 gpurun_out/ft_$w.err; exit 1; }
grep "^sweep" gpurun_out/ft_$w.err | tail -12
