# round 4, session 20: the N > 1 bench path rehearsed on one GPU (one-rank RCCL communicator):
# partition-first (general) and presorted exchanges, C4 and C3 shapes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > gpurun_out/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' gpurun_out/$name.txt | cut -c1-400
  return $rc
}
step r4s20_sh_c4 240 python -u bench.py --sharded --steps 5 --warmup 2 --no-cpu-baseline --no-traffic && \
step r4s20_sh_c4_pre 240 python -u bench.py --sharded --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --opt exchange=presorted && \
step r4s20_sh_c3 240 python -u bench.py --sharded --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-traffic && \
step r4s20_steps8 240 python -u tools/bench_sharded_steps.py --ranks 8
