#!/bin/bash
# rocprofv3 passes over a short bench run of one workload: kernel trace + stats,
# then one PMC pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a
# pass on gfx950; 8 SQ counters per pass).  Each pass runs bench.py itself after
# `--` (no launcher hop) under its own time limit.
# Usage (GPU box): [LABEL=<summary name>] bash tools/pmc.sh <tag> [workload] [extra bench args...]
#   -> gpurun_out/prof_<tag>/{trace,fetch,write,sq,sq2}/...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=${1:-r02}; wl=${2:-C2}; shift 2; extra="$@"
out=gpurun_out/prof_$tag
mkdir -p $out
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d $out/$name -o run -- \
    python3 bench.py --workload $wl $extra --steps 5 --warmup 2 --profile-steps 2 --no-cpu-baseline \
    > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $out/$name.log; exit $rc; fi
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT
python3 tools/pmc_summary.py $out ${LABEL:-${tag}_$wl}
