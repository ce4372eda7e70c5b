#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group) over tools/lab.py variants.
# usage: bash tools/pmc.sh TAG "variants" [lib]
set -u
TAG=$1; V=$2; LIB=${3:-liblab.so}
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS GRBM_COUNT SQ_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_BUSY_max TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $G -d gpurun_out/${TAG}_pmc$i -o p --output-format csv -- python3 tools/lab.py --lib $LIB --rounds 1 --variants $V > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "pmc group $i failed"; exit 1; }
done
echo pmc done
