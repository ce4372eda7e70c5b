#!/bin/bash
# Same-box A/B of the u32 keys-only pass kernel (GRS_U32_PASS) inside bench.py.
set -u
mkdir -p gpurun_out
for r in 1 2; do
for p in v3 ar1024 ar512x72; do
  GRS_U32_PASS=$p timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/abp_${p}_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/abp_${p}_$r.log').read().strip().splitlines()[-1]); print('$p r$r', d['value'], d['phases_ms'])"
done; done
