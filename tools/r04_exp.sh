#!/bin/bash
# Round-4 experiment batch: sweep variants (tools/r04_sweep.sh arguments) on C2 and
# C2 P_HOT, then (SWEEP_ALL=1 semantics for the ALL list) C3/C5, then the fix-up
# sweep traces of C2 and P_HOT.  Usage: ALL="v1 v2" bash tools/r04_exp.sh variants...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/r04_sweep.sh "$@" || exit 1
for v in $ALL; do SWEEP_ALL=1 bash tools/r04_sweep.sh "$v" | grep -E '_C3|_C5|FAILED' || exit 1; done
for w in C2 C2hot; do
  extra=""; [ "$w" = "C2hot" ] && extra="--params hot"
  MM_FIX_TRACE=1 MM_FIX_TRACE_DUMP=gpurun_out/fixdump_$w.bin timeout -k 10 200 python -u bench.py --workload C2 $extra \
    --steps 1 --warmup 1 --profile-steps 1 --no-cpu-baseline > gpurun_out/ft_$w.json 2> gpurun_out/ft_$w.err \
    || { tail -5 gpurun_out/ft_$w.err; exit 1; }
  echo "fix trace $w"; python tools/fix_fit.py gpurun_out/fixdump_$w.bin
done
