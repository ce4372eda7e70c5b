#!/bin/bash
# A/B of the record passes for u32 pairs (--opt records=0|1|2) on one box: C3 (XL tiles) and 2^26 /
# 2^24 pairs (big tiles; v4 / persistent v6) bench lines, interleaved.
mkdir -p gpurun_out
for rep in 1 2; do
  for n in 268435456 67108864 16777216; do
    for r in 0 1 2; do
      timeout -k 10 200 python -u bench.py --opt records=$r --config c3 --n $n --steps 20 --no-cpu-baseline > gpurun_out/abrec_${n}_${r}_${rep}.log 2>&1 || exit $?
      tail -1 gpurun_out/abrec_${n}_${r}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n=$n records=$r', d['value'], d['roofline']['kernel'], d['phases_ms'])"
    done
  done
done
