#!/bin/bash
# A/B of the run-line nontemporal store policy inside the sort: libgrs.so (default stores) vs
# tools/libgrs_nt.so (built with -DGRS_RUN_NT_STORES=1), interleaved, same box; then the parity
# tests of the 8-bit passes on the NT build
set -u
mkdir -p gpurun_out
B=/tmp/ntrepo
rm -rf $B && mkdir -p $B && tar --exclude=./gpurun_out -cf - . | (cd $B && tar xf -)
cp tools/libgrs_nt.so $B/gpuradixsort_amd/libgrs.so
for r in 1 2; do
  for cfg in ns c4 c3 c5; do
    timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/abnt_A_${cfg}_$r.json 2>/dev/null || exit 1
    (cd $B && timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-traffic --no-cpu-baseline) > gpurun_out/abnt_B_${cfg}_$r.json 2>/dev/null || exit 1
    python3 - "$cfg" "$r" <<'PY'
import json, sys
cfg, r = sys.argv[1], sys.argv[2]
a = json.loads(open(f"gpurun_out/abnt_A_{cfg}_{r}.json").read().strip().splitlines()[-1])
b = json.loads(open(f"gpurun_out/abnt_B_{cfg}_{r}.json").read().strip().splitlines()[-1])
print(f"{cfg} r{r}: default {a['value']:7.2f} Gkeys/s pass {a['roofline']['kernel_mean_ms']:.4f} ms | run-nt {b['value']:7.2f} pass {b['roofline']['kernel_mean_ms']:.4f}", flush=True)
PY
  done
done
(cd $B && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c4.py -k "not lds_lane_order" ) > gpurun_out/abnt_tests.log 2>&1
echo "NT build tests rc=$?"; tail -2 gpurun_out/abnt_tests.log
