# round 4, session 2: C2 (2^24 keys, 4-bit) -- phase stamps of the persistent 4-bit pass and the
# MALL-resident memory floor of its 8 passes (scatter_emu16)
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
step r4s2_c2stamps 200 python -u tools/lab2.py --n 16777216 --rounds 9 --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:8:256 --emu16 1024:32,512:32,256:16
