# round 4, session 21: 32-copy histogram for u64 keys (C5): GPU suite + C5 bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4s21_pytest.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline > gpurun_out/r4s21_c5.txt 2>&1
rc=$?; tail -2 gpurun_out/r4s21_pytest.txt; grep '^{' gpurun_out/r4s21_c5.txt | cut -c1-200; exit $rc
