# round 4, session 9: the replay floor of the pass's exact access pattern beside the shipped pass
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --variants p4:32:0:1024:36:1:272,p4:32:0:768:64:1:1040 --replay 1024:36:8,768:64:8,1024:48:8 > gpurun_out/r4s9_replay28.txt 2>&1 && \
timeout -k 10 300 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants p4:32:0:768:64:1:1040 --replay 768:64:8,1024:36:8 > gpurun_out/r4s9_replay30.txt 2>&1 && \
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 9 --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:8:256 --replay 1024:32:4 > gpurun_out/r4s9_replay24.txt 2>&1
rc=$?; grep -h "median\|workgroups" gpurun_out/r4s9_replay*.txt; exit $rc
