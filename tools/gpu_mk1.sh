#!/bin/bash
# k-way merge: presorted GPU tests, then the 8-rank step bench (both merges), rocprof of it
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_presorted.py > gpurun_out/mk1_tests.log 2>&1 || { tail -30 gpurun_out/mk1_tests.log; exit 1; }
tail -3 gpurun_out/mk1_tests.log
timeout -k 10 300 python -u tools/bench_presorted_steps.py --ranks 8 > gpurun_out/mk1_steps8.log 2>&1 || exit 1
cat gpurun_out/mk1_steps8.log
timeout -k 10 300 python -u tools/bench_presorted_steps.py --ranks 4 > gpurun_out/mk1_steps4.log 2>&1 || exit 1
cat gpurun_out/mk1_steps4.log
