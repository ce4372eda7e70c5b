#!/bin/bash
# Same-box A/B of XCD ranges inside bench.py (--opt xcd_ranges=0|1), interleaved, per config
set -u
for r in 1 2; do
  for c in ns c4 c2 c3 c5; do
    for x in 1 0; do
      out=$(timeout -k 10 200 python bench.py --config $c --steps 10 --no-cpu-baseline --opt xcd_ranges=$x 2>/dev/null | tail -1) || { echo "FAIL $c $x"; exit 1; }
      echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', 'xr=$x', d['value'], 'pass_ms', d['roofline']['kernel_mean_ms'], 'frac', d['roofline']['frac'], 'hist', d['phases_ms']['hist'], d['roofline']['kernel'])"
    done
  done
done
