#!/bin/bash
# Histogram grid A/B inside bench.py (GRS_HIST_GRID caps the grid; the 16-bit counter bound
# n >> 18 still applies) on C2 and C3.
mkdir -p gpurun_out
for r in 1 2; do
  for g in 64 128 256 512 1024 2048; do
    GRS_HIST_GRID=$g timeout -k 10 120 python bench.py --config c2 --no-cpu-baseline --steps 20 > gpurun_out/abh_c2_g${g}_r$r.log 2>&1 || exit 1
  done
  for g in 1024 2048 4096; do
    GRS_HIST_GRID=$g timeout -k 10 120 python bench.py --config c3 --no-cpu-baseline --steps 10 > gpurun_out/abh_c3_g${g}_r$r.log 2>&1 || exit 1
  done
done
