# round 4, session 15: tile shapes between 36K and 48K at the north star's 2^28 (pass + replay floor)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lab2.py --n 268435456 --rounds 9 --variants v4:32:0:1024:36:1:272,v4:32:0:1024:40:1:1040,v4:32:0:768:56:1:1040,v4:32:0:768:60:1:1040,v4:32:0:768:64:1:1040 --replay 1024:36:8,1024:40:8,768:56:8,768:60:8 > gpurun_out/r4s15_shapes28.txt 2>&1
rc=$?; grep -h "median" gpurun_out/r4s15_shapes28.txt; exit $rc
