set -u
mkdir -p gpurun_out
for r in 1 2; do
for cfg in "nt 2048" "default 2048" "nt 1024" "default 1024"; do
  set -- $cfg
  GRS_V3_DMA=$1 GRS_HIST_GRID=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ab_$1_$2_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$1_$2_$r.log').read().strip().splitlines()[-1]); print('$1 $2 r$r', d['value'], d['phases_ms'])"
done; done
