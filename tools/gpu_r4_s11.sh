# round 4, session 11: per-XCD ticket heads (lab OPT 134217728) on the pass and on its replay floor
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --variants v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:134218000,v4:32:0:768:64:1:1040,v4:32:0:768:64:1:134218768,v4:32:0:1024:36:1:134218008 --replay 1024:36:8:0,1024:36:8:1 > gpurun_out/r4s11_x8_28.txt 2>&1 && \
timeout -k 10 300 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040,v4:32:0:768:64:1:134218768 --replay 768:64:8:0,768:64:8:1 > gpurun_out/r4s11_x8_30.txt 2>&1 && \
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 9 --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:134217728:256,r6:32:0:1024:32:1:134217736:256 --replay 1024:32:4:0,1024:32:4:1 > gpurun_out/r4s11_x8_24.txt 2>&1
rc=$?; grep -h "median\|ticket known\|^stamps\|workgroups" gpurun_out/r4s11_x8_*.txt; exit $rc
