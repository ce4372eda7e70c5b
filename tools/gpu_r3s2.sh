#!/bin/bash
# Round-3 (session 2) evidence: parity tests, smoke, bench lines (C4 default with PMC traffic, ns,
# C2, C3, C5), rocprof kernel stats of C4 and ns.   bash tools/gpu_r3_final.sh TAG
set -u
TAG=${1:-r3s2}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "   $name rc=$rc"
  return $rc
}
run pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -1 gpurun_out/${TAG}_pytest.log
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 400 python -u bench.py || exit $?
for c in ns c2 c3 c5; do run bench_$c 400 python -u bench.py --config $c --steps 10 --no-cpu-baseline || exit $?; done
run prof_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c4 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic || exit $?
run prof_ns 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_ns -o run --output-format csv -- python3 bench.py --config ns --steps 10 --warmup 2 --no-cpu-baseline --no-traffic || exit $?
run prof_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic || exit $?
run prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-traffic || exit $?
exit 0
