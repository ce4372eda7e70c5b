#!/bin/bash
# Round-4 evidence session: GPU tests, smoke, the driver's bench line (C4 + north-star leg, PMC
# traffic, CPU baseline), bench lines of C2 / C3 / C5, rocprof kernel stats of C4, ns, C2, C3,
# the §8f extras.   bash tools/gpu_r4_final.sh TAG [PART]   (PART a: tests + smoke + bench;
# b: other configs + rocprof; default both)
set -u
TAG=${1:-r4f}
PART=${2:-ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "   $name rc=$rc"
  tail -2 "gpurun_out/${TAG}_${name}.log" | cut -c1-300
  return $rc
}
if [[ $PART == *a* ]]; then
  run pytest 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
  run bench 500 python -u bench.py || exit $?
  run extras 300 python -u tools/bench_extras.py || exit $?
fi
if [[ $PART == *b* ]]; then
  for c in c2 c3 c5; do run bench_$c 300 python -u bench.py --config $c --steps 10 --no-cpu-baseline || exit $?; done
  run prof_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c4 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-north-star || exit $?
  run prof_ns 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_ns -o run --output-format csv -- python3 bench.py --config ns --steps 10 --warmup 2 --no-cpu-baseline --no-traffic || exit $?
  run prof_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-traffic || exit $?
  run prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-traffic || exit $?
fi
exit 0
