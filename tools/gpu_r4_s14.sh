# round 4, session 14: register/shuffle bitonic stages for short segments
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out

timeout -k 10 200 python -u tools/bench_extras.py --partition-ab > gpurun_out/r4s14_bench_extras.txt 2>&1
rc=$?; tail -3 gpurun_out/r4s14_extras_tests.txt; grep op gpurun_out/r4s14_bench_extras.txt; exit $rc
