# round 4, session 5: the sharded tests (shrunk-region option range fixed), then per-CU tile
# gaps of the shipped pass shapes (lab stamps slots 10/11)
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
step r4s5_sharded 300 python -u -m pytest tests/test_gpu_sharded.py -q --timeout 120 --timeout-method thread
step r4s5_gap28 240 python -u tools/lab2.py --n 268435456 --rounds 3 --variants v4:32:0:1024:36:1:280,v4:32:0:768:64:1:1048,v6:32:0:1024:36:1:264:256
step r4s5_gap30 240 python -u tools/lab2.py --n 1073741824 --rounds 3 --variants v4:32:0:768:64:1:1048,v4:32:0:1024:36:1:280
step r4s5_gap24 240 python -u tools/lab2.py --n 16777216 --rounds 5 --variants r6:32:0:1024:32:1:8:256,r4:32:0:1024:32:1:8
