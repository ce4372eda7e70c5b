# round 4, session 28: the persistent pass with a fixed-count prefetch and the group re-polls
# waited at the loop's bottom (so the look-back's first test no longer waits for the prefetch),
# A/B against the committed library (abold/), alternating
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $secs "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc $(tail -1 gpurun_out/$name.txt | cut -c1-160)" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
F="--no-cpu-baseline --no-north-star --no-traffic --steps 30"
for r in 1 2; do
  step r4s28_c2_new$r 180 python -u bench.py --config c2 $F
  step r4s28_c2_old$r 180 python -u abold/bench.py --config c2 $F
  step r4s28_c4n24_new$r 180 python -u bench.py --config c4 --n 16777216 $F
  step r4s28_c4n24_old$r 180 python -u abold/bench.py --config c4 --n 16777216 $F
  step r4s28_c4n25_new$r 180 python -u bench.py --config c4 --n 33554432 $F
  step r4s28_c4n25_old$r 180 python -u abold/bench.py --config c4 --n 33554432 $F
done
