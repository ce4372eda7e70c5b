# round 4, session 3: the error-path tests alone (the u64 case raised an illegal access inside
# the full suite in session 2 but not in isolation), then the full GPU suite, then phase stamps
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
  if grep -q "illegal memory access\|hipErrorIllegalAddress" gpurun_out/$name.txt; then echo "GPU fault in $name: stopping" >&2; exit 99; fi
  return 0
}
step r4s3_errors 300 python -u -m pytest tests/test_gpu_errors.py -v --timeout 120 --timeout-method thread
step r4s3_pytest 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step r4s3_stamps28 240 python -u tools/lab2.py --n 268435456 --rounds 5 --variants v4:32:0:1024:36:1:280,v4:32:0:768:64:1:1048,v6:32:0:1024:36:1:264:256,v6:32:0:1024:36:1:524568:256
step r4s3_stamps30 240 python -u tools/lab2.py --n 1073741824 --rounds 3 --variants v4:32:0:768:64:1:1048,v4:32:0:1024:36:1:280
