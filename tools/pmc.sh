#!/bin/bash
# PMC passes over tools/blockbench.py (one counter group per pass; no tracing
# domains beside --kernel-trace, per the pool rules).  usage: tools/pmc.sh TAG [blockbench args]
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- python3 ${PMC_SCRIPT:-tools/blockbench.py} "$@" > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG
