#!/bin/bash
# C2 (2^24 u32 keys, 4-bit digits) experiments: histogram grid, kernel durations, pass stamps.
#   bash tools/exp_c2.sh TAG
TAG=${1:-c2x}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" > gpurun_out/${TAG}_${name}.log 2>&1; local rc=$?; echo "   rc=$rc" >&2; return $rc; }
for g in 64 128 256 512; do
  GRS_HIST2_GRID=$g run bench_g$g 120 python -u bench.py --config c2 --no-cpu-baseline || exit $?
  tail -1 gpurun_out/${TAG}_bench_g$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('grid $g', d['value'], d['phases_ms'])" >&2
done
run prof_c2 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit $?
run lab_r6 200 python3 -u tools/lab2.py --n 16777216 --rounds 9 --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:8:256,r6:32:0:512:32:2:0:512,r6:32:0:256:32:4:0:1024 || exit $?
tail -8 gpurun_out/${TAG}_lab_r6.log >&2
