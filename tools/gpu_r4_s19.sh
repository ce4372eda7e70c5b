# round 4, session 19: the §8f extras including the record sort
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_extras.py > gpurun_out/r4s22_bench_extras.txt 2>&1
rc=$?; grep op gpurun_out/r4s22_bench_extras.txt; tail -3 gpurun_out/r4s22_bench_extras.txt; exit $rc
