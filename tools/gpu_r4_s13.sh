# round 4, session 13: the one-pass scan and the short-segment path in the library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_extras.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s13_extras_tests.txt 2>&1 && \
timeout -k 10 120 python -u tools/ab_scan.py > gpurun_out/r4s13_scan.txt 2>&1 && \
timeout -k 10 200 python -u tools/bench_extras.py > gpurun_out/r4s13_bench_extras.txt 2>&1
rc=$?; tail -3 gpurun_out/r4s13_extras_tests.txt; grep "n=" gpurun_out/r4s13_scan.txt; cat gpurun_out/r4s13_bench_extras.txt | grep op; exit $rc
