#!/bin/bash
# Round-4 probe: per-launch traces of C2 (P_FULL, P_HOT) and comp_rms ablations.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/ktrace.sh r04a C2 > gpurun_out/kt_r04a_C2.txt 2>&1 || { cat gpurun_out/kt_r04a_C2.txt | tail; exit 1; }
bash tools/ktrace.sh r04b C2hot > gpurun_out/kt_r04b_C2hot.txt 2>&1 || exit 1
bash tools/fix_trace.sh C2 > gpurun_out/ft_r04_C2.txt 2>&1 || exit 1
bash tools/ablate.sh comp_rms comp_describe comp_pass0 comp_fix comp_apply
