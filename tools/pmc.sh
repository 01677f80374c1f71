#!/bin/bash
# rocprofv3 passes over a short C2 bench run: kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# Usage (on the GPU box): bash tools/pmc.sh <tag>   -> gpurun_out/prof_<tag>/...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=${1:-r01}
out=gpurun_out/prof_$tag
mkdir -p $out
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" --output-format csv -d $out/$name -o run -- \
    python3 bench.py --steps 5 --warmup 2 --profile-steps 2 --no-cpu-baseline > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $out/$name.log; exit $rc; fi
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
find $out -name "*.csv" | sort
