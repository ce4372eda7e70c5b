#!/bin/bash
# Round-2 A/B (b): 4-bit pass shapes for C2 (tools/lab2.py, 2^24 keys), and the big-pass
# variants (GRS_PASS_VARIANT) for C3 / C5 inside bench.py, two interleaved rounds.
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/lab2.py --n 16777216 --check --rounds 15 --variants \
r4:32:0:256:16:4:0,r4:32:0:256:16:4:512,r4:32:0:256:16:4:16,r4:32:0:512:16:2:0,r4:32:0:512:16:2:512,\
r4:32:0:1024:16:1:0,r4:32:0:1024:16:1:512,r4:32:0:1024:8:1:0,r4:32:0:1024:8:1:512,r4:32:0:256:32:4:0,\
r4:32:0:256:32:4:512,r4:32:0:512:32:2:0,r4:32:0:512:32:2:512,r4:32:0:1024:32:1:0,r4:32:0:1024:32:1:512,\
r4:32:0:256:8:8:0,r4:32:0:256:8:8:512,r4:32:0:128:16:8:0,r4:32:0:128:16:8:512,r4:32:0:512:8:4:512 \
  > gpurun_out/ab3_c2lab.log 2>&1 || exit 1
for r in 1 2; do
  for c in c3 c5; do
    for v in 0 1 2; do
      GRS_PASS_VARIANT=$v timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 10 > gpurun_out/ab3_${c}_v${v}_r$r.log 2>&1 || exit 1
    done
  done
done
