#!/bin/bash
# SQ counters of the pass kernel at the ns config (2^28 u32 keys): where a tile's cycles go.
#   bash tools/pmc_sq.sh TAG [bench args...]
set -u
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/${TAG}_sq$i -o p --output-format csv -- python3 bench.py "$@" > gpurun_out/${TAG}_sq$i.log 2>&1
  echo "sq$i rc=$?"
done
python3 tools/pmc_kernels.py gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2 > gpurun_out/${TAG}_sq_summary.txt 2>&1 || true
