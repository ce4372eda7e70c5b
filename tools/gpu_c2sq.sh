#!/bin/bash
# C2 (2^24 keys, 4-bit): SQ counters of the persistent pass and a kernel-trace timeline of the
# sort (per-kernel durations and the gaps between consecutive launches)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c2tl
bash tools/pmc_sq.sh c2 --config c2 --steps 3 --warmup 1 --no-traffic --no-cpu-baseline || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/c2tl -o tl -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/c2tl/bench.log 2>&1 || exit 1
