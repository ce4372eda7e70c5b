#!/bin/bash
# A/B of the upfront histogram kernels inside bench.py (GRS_HIST=1 round-1 layout, 2 = hist2),
# then a grid sweep of hist2 (GRS_HIST2_GRID).  tools/ab_hist2.sh TAG
TAG=${1:-abh2}
mkdir -p gpurun_out
b() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 ${CFG:+--config $CFG} > gpurun_out/${TAG}_${name}.log 2>&1 || { echo "FAIL $name" >&2; exit 1; }; }
for r in 1 2; do
  for c in c4 c2 c3 c5; do
    for h in 1 2; do CFG=$c b ${c}_h${h}_r$r GRS_HIST=$h; done
  done
done
for g in 256 512 1024; do CFG=c2 b c2_g${g} GRS_HIST2_GRID=$g; done
for g in 512 1024 1536 2048 3072; do CFG=c4 b c4_g${g} GRS_HIST2_GRID=$g; done
