# round 4, session 6: digit waves' prefetch behind their stores (lab OPT 2048)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:524560:256,v6:32:0:1024:36:1:526608:256,v6:32:0:1024:36:1:526616:256 > gpurun_out/r4s6_pf28.txt 2>&1 && \
timeout -k 10 240 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:526608:256 > gpurun_out/r4s6_pf30.txt 2>&1
rc=$?; tail -12 gpurun_out/r4s6_pf28.txt; tail -5 gpurun_out/r4s6_pf30.txt; exit $rc
