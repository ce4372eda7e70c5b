#!/bin/bash
# A/B of the record passes for u32 pairs (GRS_RECORDS) on one box: C3 bench lines, interleaved.
mkdir -p gpurun_out
for rep in 1 2 3; do
  for r in 0 1; do
    GRS_RECORDS=$r timeout -k 10 200 python -u bench.py --config c3 --steps 20 --no-cpu-baseline > gpurun_out/abrec_${r}_${rep}.log 2>&1 || exit $?
    tail -1 gpurun_out/abrec_${r}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('records=$r', d['value'], d['phases_ms'])"
  done
done
