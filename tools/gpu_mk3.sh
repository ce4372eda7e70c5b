#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in 0 1 2 3; do
  mkdir -p gpurun_out/mk3_$d
  GRS_MK_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mk3_$d -o p -- python3 tools/bench_presorted_steps.py --ranks 8 --reps 3 > gpurun_out/mk3_$d/steps.log 2>&1 || exit 1
done
