#!/bin/bash
# One GPU-box session: parity tests, bench lines for every config, rocprof summary.
# usage (via gpurun): bash tools/gpu_session.sh [tag]
set -u
TAG=${1:-s}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run pytest 900 python -m pytest tests -m gpu -q -p no:cacheprovider
rc=$?
[ $rc -gt 1 ] && exit $rc
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 300 python bench.py || exit $?
for c in c2 c3 c5; do run bench_$c 300 python bench.py --config $c --steps 10 --no-cpu-baseline || exit $?; done
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit $?
exit 0
