# round 4, session 10: two-round 1024-thread tiles (longer runs, 16 waves) against big / XL
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=v4:32:0:1024:36:1:272,v4:32:0:768:64:1:1040,v4:32:0:1024:48:1:1040,v4:32:0:1024:48:1:1296,v4:32:0:1024:56:1:1296,v4:32:0:1024:62:1:1296,v4:32:0:1024:44:1:1296
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --variants $V > gpurun_out/r4s10_tr28.txt 2>&1 && \
timeout -k 10 300 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants $V > gpurun_out/r4s10_tr30.txt 2>&1
rc=$?; grep -h "median" gpurun_out/r4s10_tr*.txt; exit $rc
