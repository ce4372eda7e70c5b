#!/bin/bash
# kernel stats of the 8-rank presorted steps (k-way merge kernels)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mk2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mk2 -o mk2 -- python3 tools/bench_presorted_steps.py --ranks 8 --reps 3 > gpurun_out/mk2/steps.log 2>&1 || exit 1
f=$(find gpurun_out/mk2 -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -30
