# round 4, session 33: the partition's digit histogram with a resident grid (new) against the
# committed library (abold/), alternating; then the kernel stats of the new one
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep '"op"' gpurun_out/$name.txt | cut -c1-140)" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
for r in 1 2 3; do
  step r4s33_new$r 120 python -u tools/prof_partition.py
  step r4s33_old$r 120 python -u abold/tools/prof_partition.py
done
step r4s33_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s33_prof -o run --output-format csv -- python3 tools/prof_partition.py
