#!/bin/bash
# ns: persistent pass / XL / tile options inside the sort, 2 rounds interleaved
set -u
for r in 1 2; do
  for o in "" "--opt pass=v6" "--opt xl=1"; do
    echo "== $o"
    timeout -k 10 120 python -u bench.py --config ns --steps 10 --no-cpu-baseline $o | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_mean_ms'], d['phases_ms'])" || exit $?
  done
done
