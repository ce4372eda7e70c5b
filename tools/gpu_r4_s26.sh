# round 4, session 26: do scalar glc loads observe another XCD's status store?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/smem_probe.py > gpurun_out/r4s26_smem.txt 2>&1
rc=$?; cat gpurun_out/r4s26_smem.txt | grep -v amdgpu.ids; exit $rc
