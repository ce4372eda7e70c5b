#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE / L2 hit counters, one rocprofv3 pass each) of
# tools/lab.py variants.  usage: bash tools/pmc_traffic.sh TAG "variants" [lib]
set -u
TAG=$1; V=$2; LIB=${3:-liblab.so}
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $G -d gpurun_out/${TAG}_pmc$i -o p --output-format csv -- python3 tools/lab.py --lib $LIB --rounds 1 --copy --variants $V > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "pmc group $i failed"; exit 1; }
done
python3 tools/pmc_summary.py $TAG
