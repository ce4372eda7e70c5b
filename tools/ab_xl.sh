#!/bin/bash
# Same-box A/B of the two-round XL tiles inside bench.py: --opt xl=1 (forced) vs 0 (never).
TAG=${1:-abxl}
mkdir -p gpurun_out
for r in 1 2; do
  for c in c4 c3 c5; do
    for x in 0 1; do
      timeout -k 10 200 python bench.py --opt xl=$x --config $c --no-cpu-baseline --steps 10 > gpurun_out/${TAG}_${c}_x${x}_r$r.log 2>&1 || { echo "FAIL $c $x" >&2; exit 1; }
    done
  done
done
