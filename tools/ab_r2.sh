#!/bin/bash
# Same-box A/B of pass variants inside bench.py (round 2): u32 variants (GRS_U32_PASS) on C4,
# nontemporal tile loads (GRS_PASS_NT) on C3 / C5, and C2.  Two interleaved rounds.
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1 2 3 4 5 6; do
    GRS_U32_PASS=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab2_u$v_$r.log 2>&1 || exit 1
    mv gpurun_out/ab2_u$v_$r.log gpurun_out/ab2_u${v}_r$r.log
  done
  for c in c3 c5; do
    for nt in 0 1; do
      GRS_PASS_NT=$nt timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 10 > gpurun_out/ab2_${c}_nt${nt}_r$r.log 2>&1 || exit 1
    done
  done
  timeout -k 10 120 python bench.py --config c2 --no-cpu-baseline --steps 20 > gpurun_out/ab2_c2_r$r.log 2>&1 || exit 1
done
