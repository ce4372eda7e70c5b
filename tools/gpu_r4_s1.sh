# round 4, session 1: GPU tests of the stripped pass + error-path tests, the boundary-line
# hand-off emulation, and a first bench of the two-leg bench.py.  A step that times out, faults
# or aborts ends the script (rc >= 124 or a signal); test failures (rc 1) do not.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $secs "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -3 gpurun_out/$name.txt >&2
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
step r4s1_pytest 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r4s1_emu28 240 python -u tools/lab2.py --n 268435456 --rounds 7 --variants v4:32:0:1024:36:1:272 --emu 1024:36:0:150000,1024:36:1:150000,1024:36:3:150000,1024:36:5:150000,1024:48:3:150000 --emu-handoff 1024:36:0:150000,1024:36:1:150000,1024:36:2:150000,1024:48:0:150000,1024:48:1:150000
step r4s1_emu30 300 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040 --emu 1024:36:0:150000,1024:36:3:150000,1024:36:5:150000,1024:48:3:150000 --emu-handoff 1024:36:0:150000,1024:36:1:150000,1024:48:0:150000
step r4s1_p4 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants p4:32:0:1024:36:1:272,p4:32:0:1024:36:1:336,v4:32:0:1024:36:1:272,p4:32:0:768:64:1:1040,p4:32:0:768:64:1:1104
step r4s1_p4gw2 200 python -u tools/lab2.py --n 268435456 --rounds 9 --lib4 gw2 --variants p4:32:0:1024:36:1:272,p4:32:0:768:64:1:1040
step r4s1_p4gw4 200 python -u tools/lab2.py --n 268435456 --rounds 9 --lib4 gw4 --variants p4:32:0:1024:36:1:272
step r4s1_p4_30 300 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants p4:32:0:768:64:1:1040,p4:32:0:768:64:1:1104,p4:64:0:768:44:1:1040,p4:64:0:768:44:1:1104
step r4s1_bench 400 python -u bench.py
