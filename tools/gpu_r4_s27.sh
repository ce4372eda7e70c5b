# round 4, session 27: the look-back's own-group re-polls through scalar loads (OPT 4) in the
# persistent pass (where vector re-polls queue behind the prefetch) and in v4; stamps (OPT 8)
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
step r4s27_probe 120 python -u tools/smem_probe.py
step r4s27_stamps28 240 python -u tools/lab2.py --n 268435456 --rounds 3 --variants v6:32:0:1024:36:1:264:256,v6:32:0:1024:36:1:268:256,v4:32:0:1024:36:1:280,v4:32:0:1024:36:1:284
step r4s27_time28 240 python -u tools/lab2.py --n 268435456 --rounds 7 --variants v6:32:0:1024:36:1:256:256,v6:32:0:1024:36:1:260:256,v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:276
step r4s27_time24 240 python -u tools/lab2.py --n 16777216 --rounds 7 --variants v6:32:0:1024:36:1:256:256,v6:32:0:1024:36:1:260:256,v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:276
