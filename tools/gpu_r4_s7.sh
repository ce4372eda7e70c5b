# round 4, session 7: C2 (2^24, 4-bit) -- where a pass's time goes outside its tiles; one-tile-per-CU shapes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 5 --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:8:256,v6:32:0:1024:36:1:264:256 > gpurun_out/r4s8_c2.txt 2>&1
rc=$?; grep -A4 "median\|^stamps" gpurun_out/r4s8_c2.txt | grep -v "ticket known"; exit $rc
