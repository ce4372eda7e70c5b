#!/bin/bash
# Round-end GPU session: parity tests, smoke, bench lines (C4 default, 256M u32, C2, C3, C5),
# extras, rocprof kernel stats and PMC traffic of the headline config.
# usage (via gpurun): bash tools/gpu_final.sh TAG
set -u
TAG=${1:-fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit $?
run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
run pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
python3 tools/bench_pmc.py ${TAG} c4 134217728 > gpurun_out/${TAG}_pmc.log 2>&1; echo "pmc parse rc=$?"
run bench 300 python bench.py || exit $?
run bench_256m 300 python bench.py --n 268435456 --steps 10 --no-cpu-baseline || exit $?
for c in c2 c3 c5; do run bench_$c 300 python bench.py --config $c --steps 10 --no-cpu-baseline || exit $?; done
run extras 200 python tools/bench_extras.py || exit $?
exit 0
