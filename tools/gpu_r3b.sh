#!/bin/bash
# round-3 session-2 check: full GPU suite, then bench lines (no traffic) for c2 / ns / c4 and a
# kernel trace of C2 sorts (launch gaps without the per-phase event ring)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3b/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3b/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for cfg in c2 ns c4; do
  timeout -k 10 300 python bench.py --config $cfg --no-traffic --no-cpu-baseline > gpurun_out/r3b/bench_$cfg.json 2> gpurun_out/r3b/bench_$cfg.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3b/bench_$cfg.json').read().strip().splitlines()[-1]);print('$cfg', d['value'], d['unit'], d['roofline']['frac'], d['phases_ms'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3b/c2tl -o tl -- python3 tools/exp_events.py --configs c2 --steps 10 > gpurun_out/r3b/c2tl.log 2>&1 || exit 1
