#!/bin/bash
# Same-box A/B of the pass kernel inside bench.py: --opt pass=v4 (one tile per workgroup) vs v6
# (persistent, next-tile prefetch), every config, two interleaved rounds.  tools/ab_pass.sh TAG
TAG=${1:-abp}
mkdir -p gpurun_out
for r in 1 2; do
  for c in c4 c2 c3 c5; do
    for v in v4 v6; do
      timeout -k 10 200 python bench.py --opt pass=$v --no-cpu-baseline --steps 10 --config $c > gpurun_out/${TAG}_${c}_${v}_r$r.log 2>&1 || { echo "FAIL $c $v" >&2; exit 1; }
    done
  done
done
