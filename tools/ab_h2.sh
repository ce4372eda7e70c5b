#!/bin/bash
# A/B: histogram grid of one (libgrs.so) vs two (tools/libgrs_h2.so) 512-thread blocks per CU for
# sorts of <= 2^25 keys (C2), interleaved; plus the sharded bench paths on one GPU
set -u
mkdir -p gpurun_out
B=/tmp/h2repo
rm -rf $B && mkdir -p $B && tar --exclude=./gpurun_out -cf - . | (cd $B && tar xf -)
cp tools/libgrs_h2.so $B/gpuradixsort_amd/libgrs.so
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-traffic --no-cpu-baseline > gpurun_out/abh2_A_$r.json 2>/dev/null || exit 1
  (cd $B && timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-traffic --no-cpu-baseline) > gpurun_out/abh2_B_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
a=json.loads(open('gpurun_out/abh2_A_$r.json').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/abh2_B_$r.json').read().strip().splitlines()[-1])
print('r$r one block/CU', a['value'], a['phases_ms']['hist'], '| two', b['value'], b['phases_ms']['hist'])"
done
timeout -k 10 200 python bench.py --sharded --steps 5 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/sh1.json 2>gpurun_out/sh1.err; echo "sharded rc=$?"; tail -c 700 gpurun_out/sh1.json
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-traffic --no-cpu-baseline > gpurun_out/sh2.json 2>gpurun_out/sh2.err; echo "torchrun rc=$?"; tail -c 300 gpurun_out/sh2.json
