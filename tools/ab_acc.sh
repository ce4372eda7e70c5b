#!/bin/bash
# A/B of the group-accumulator read-back (libgrs.so, the default) vs the returning add
# (tools/libgrs_noacc.so, built with -DGRS_ACC_READBACK=0), interleaved on one box; then the
# whole GPU suite on the default build
set -u
mkdir -p gpurun_out
B=/tmp/noaccrepo
rm -rf $B && mkdir -p $B && tar --exclude=./gpurun_out -cf - . | (cd $B && tar xf -)
cp tools/libgrs_noacc.so $B/gpuradixsort_amd/libgrs.so
for r in 1 2; do
  for cfg in ns c4 c3 c5; do
    timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/abacc_A_${cfg}_$r.json 2>/dev/null || exit 1
    (cd $B && timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-traffic --no-cpu-baseline) > gpurun_out/abacc_B_${cfg}_$r.json 2>/dev/null || exit 1
    python3 - "$cfg" "$r" <<'PY'
import json, sys
cfg, r = sys.argv[1], sys.argv[2]
a = json.loads(open(f"gpurun_out/abacc_A_{cfg}_{r}.json").read().strip().splitlines()[-1])
b = json.loads(open(f"gpurun_out/abacc_B_{cfg}_{r}.json").read().strip().splitlines()[-1])
print(f"{cfg} r{r}: readback(A) {a['value']:7.2f} Gkeys/s pass {a['roofline']['kernel_mean_ms']:.4f} ms | no-readback(B) {b['value']:7.2f} pass {b['roofline']['kernel_mean_ms']:.4f}", flush=True)
PY
  done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/abacc_tests.log 2>&1
echo "default build: GPU tests rc=$?"; tail -2 gpurun_out/abacc_tests.log
