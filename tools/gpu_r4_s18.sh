# round 4, session 18: C2's persistent pass with static tiles under a cooperative launch (no ticket)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 15 --check --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:2:256,r6:32:0:1024:32:1:10:256,r6:32:0:1024:32:1:8:256 > gpurun_out/r4s18_static.txt 2>&1
rc=$?; grep -h "median\|check\|^stamps\|workgroups\|err=" gpurun_out/r4s18_static.txt | head -30; exit $rc
