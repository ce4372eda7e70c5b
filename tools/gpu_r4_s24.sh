# round 4, session 24: kernel trace of C2 sorts (gaps between the 9 launches of a sort)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4s24_c2trace -o run -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-traffic > gpurun_out/r4s24_c2trace.log 2>&1
rc=$?; ls gpurun_out/r4s24_c2trace/*/ 2>/dev/null | head; exit $rc
