# round 4, session 2: GPU tests after the fold revert, the shipped kernel beside the lab copy,
# C2 phase stamps + its MALL-resident memory floor, and the two-leg bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $secs "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -3 gpurun_out/$name.txt >&2
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step r4s2_pytest 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step r4s2_p4 200 python -u tools/lab2.py --n 268435456 --rounds 9 --variants p4:32:0:1024:36:1:272,v4:32:0:1024:36:1:272,p4:32:0:768:64:1:1040,v4:32:0:768:64:1:1040
step r4s2_c2 200 python -u tools/lab2.py --n 16777216 --rounds 9 --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:8:256 --emu16 1024:32,512:32,256:16
step r4s2_bench 400 python -u bench.py
