#!/bin/bash
# Round-2 GPU session: parity tests, then the benches (C4 default + C2/C3/C5), then profiles.
#   tools/gpu_r2.sh TAG [tests|bench|prof|all]
TAG=${1:-r2}
WHAT=${2:-all}
mkdir -p gpurun_out
run() { local name=$1 secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" > gpurun_out/${TAG}_${name}.log 2>&1; local rc=$?; echo "   rc=$rc" >&2; return $rc; }
if [[ $WHAT == tests || $WHAT == all ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
  tail -1 gpurun_out/${TAG}_pytest_gpu.log >&2
fi
if [[ $WHAT == bench || $WHAT == all ]]; then
  run bench 300 python -u bench.py || exit $?
  tail -1 gpurun_out/${TAG}_bench.log >&2
  for c in c2 c3 c5; do run bench_$c 200 python -u bench.py --config $c --no-cpu-baseline || exit $?; done
fi
if [[ $WHAT == prof || $WHAT == all ]]; then
  run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit $?
fi
