#!/bin/bash
# Memory-pipeline counter passes (TA / TCP / TD) over a short bench run of one
# workload, one pass per block group, each under its own time limit.
# Usage (GPU box): bash tools/pmc_mem.sh <tag> [workload] [extra bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=${1:-mem}; wl=${2:-C2}; shift 2; extra="$@"
out=gpurun_out/prof_$tag
mkdir -p $out
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d $out/$name -o run -- \
    python3 bench.py --workload $wl $extra --steps 3 --warmup 2 --profile-steps 1 --no-cpu-baseline \
    > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/$name.log; exit $rc; }
  return 0
}
run ta1 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum
run ta2 --pmc TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum
run tcp --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
run td --pmc TD_TD_BUSY_sum TD_TC_STALL_sum
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT
