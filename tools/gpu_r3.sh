#!/bin/bash
# Round-3 GPU session (run through gpurun): each step under its own time limit, chained so
# that the first failure ends the session.
#   bash tools/gpu_r3.sh TAG STEP [STEP ...]
# steps: tests smoke bench ns c2 c3 c5 prof_ns prof_c4 pmc_ns pmc_c4 extras
set -u
TAG=${1:-r3}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "   $name rc=$rc"
  tail -2 "gpurun_out/${TAG}_${name}.log" | cut -c1-400
  return $rc
}
prof() {  # name, timeout, bench args...
  local name=$1 to=$2; shift 2
  run "$name" "$to" rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_${name}" -o run \
    --output-format csv -- python3 bench.py "$@"
}
pmc() {  # name, counter, bench args...
  local name=$1 ctr=$2; shift 2
  run "$name" 120 rocprofv3 --pmc "$ctr" -d "gpurun_out/${TAG}_${name}" -o p --output-format csv \
    -- python3 bench.py "$@"
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $? ;;
    tests_v) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 300 python -u bench.py || exit $? ;;
    ns|c2|c3|c5|c4) run bench_$step 300 python -u bench.py --config $step --steps 10 --no-cpu-baseline || exit $? ;;
    prof_ns) prof prof_ns 300 --config ns --steps 10 --warmup 2 --no-cpu-baseline || exit $? ;;
    prof_c4) prof prof_c4 300 --steps 10 --warmup 2 --no-cpu-baseline || exit $? ;;
    prof_c2) prof prof_c2 300 --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit $? ;;
    pmc_ns) pmc pmc_ns_fetch FETCH_SIZE --config ns --steps 2 --warmup 1 --no-cpu-baseline || exit $?
            pmc pmc_ns_write WRITE_SIZE --config ns --steps 2 --warmup 1 --no-cpu-baseline || exit $? ;;
    pmc_c4) pmc pmc_c4_fetch FETCH_SIZE --steps 2 --warmup 1 --no-cpu-baseline || exit $?
            pmc pmc_c4_write WRITE_SIZE --steps 2 --warmup 1 --no-cpu-baseline || exit $? ;;
    extras) run extras 200 python tools/bench_extras.py || exit $? ;;
    *) if [[ -f "$step" ]]; then run "$(basename "$step" .sh)" 600 bash "$step" || exit $?;
       else echo "unknown step $step"; exit 2; fi ;;
  esac
done
exit 0
