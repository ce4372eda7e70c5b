#!/bin/bash
# Same-box A/B of the u32 keys-only pass kernels across sizes (GRS_U32_PASS), 8- and 4-bit.
set -u
mkdir -p gpurun_out
for n in 16777216 33554432 67108864 134217728; do
for p in v3 ar512x72; do
  GRS_U32_PASS=$p timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --n $n > gpurun_out/abs_${p}_$n.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/abs_${p}_$n.log').read().strip().splitlines()[-1]); print('$p $n rb8', d['value'], d['phases_ms']['pass_mean'])"
done; done
for n in 16777216 67108864; do
for p in v3 ar512x72; do
  GRS_U32_PASS=$p timeout -k 10 120 python bench.py --config c2 --no-cpu-baseline --steps 20 --n $n > gpurun_out/abs4_${p}_$n.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/abs4_${p}_$n.log').read().strip().splitlines()[-1]); print('$p $n rb4', d['value'], d['phases_ms']['pass_mean'])"
done; done
