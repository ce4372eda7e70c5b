#!/bin/bash
# Same-box A/B of the u32 keys pass tile inside bench.py: GRS_XL=1 (48K two-round tiles) vs 0.
TAG=${1:-abxl}
mkdir -p gpurun_out
for r in 1 2 3; do
  for x in 0 1; do
    GRS_XL=$x timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${TAG}_c4_x${x}_r$r.log 2>&1 || { echo "FAIL c4 $x" >&2; exit 1; }
  done
done
for x in 0 1; do
  GRS_XL=$x timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --n 268435456 > gpurun_out/${TAG}_n28_x${x}.log 2>&1 || exit 1
done
