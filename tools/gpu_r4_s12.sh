# round 4, session 12: single-pass scan vs reduce-then-scan
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ab_scan.py > gpurun_out/r4s12_scan.txt 2>&1
rc=$?; cat gpurun_out/r4s12_scan.txt | grep -v amdgpu.ids; exit $rc
