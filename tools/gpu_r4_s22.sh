# round 4, session 22: few long segments through key sort + one partition pass by segment
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_extras.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s22_extras_tests.txt 2>&1 && \
timeout -k 10 300 python -u tools/bench_extras.py > gpurun_out/r4s22_bench_extras.txt 2>&1
rc=$?; tail -2 gpurun_out/r4s22_extras_tests.txt; grep segmented gpurun_out/r4s22_bench_extras.txt; exit $rc
