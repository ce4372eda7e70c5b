# round 4, session 25: the GPU suite twice in a row (flakiness check before round end)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s25_pytest1.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s25_pytest2.txt 2>&1
rc=$?; tail -1 gpurun_out/r4s25_pytest1.txt; tail -1 gpurun_out/r4s25_pytest2.txt; exit $rc
