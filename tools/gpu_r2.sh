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
if [[ $WHAT == pmc || $WHAT == all ]]; then
  export TMPDIR=/tmp
  run pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
  run pmc_write 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
  run pmc_cfetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_cfetch -o p --output-format csv -- python3 tools/lab2.py --rounds 1 --variants v4:32:0:1024:36:1:272 --emu 1024:36:0:150000 || exit $?
  run pmc_cwrite 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_cwrite -o p --output-format csv -- python3 tools/lab2.py --rounds 1 --variants v4:32:0:1024:36:1:272 --emu 1024:36:0:150000 || exit $?
  run pmc_sum 60 python3 tools/bench_pmc.py ${TAG} c4 1073741824 gpurun_out/${TAG}_traffic_c4.json || exit $?
  run bench_traffic 300 python -u bench.py --traffic-json gpurun_out/${TAG}_traffic_c4.json || exit $?
  tail -1 gpurun_out/${TAG}_bench_traffic.log >&2
fi
if [[ $WHAT == prof || $WHAT == all ]]; then
  run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit $?
fi
