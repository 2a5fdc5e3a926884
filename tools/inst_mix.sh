#!/bin/bash
# Dynamic instruction mix of the network's own kernels (one PMC pass over the
# bench command): SALU / SMEM / branch / VALU / MFMA / LDS / VMEM instructions
# and waves, per kernel -> gpurun_out/imix_<TAG>/summary.txt.  One wave issues at
# most one instruction per ~4 cycles, so the per-band instruction count of a
# stack kernel's wave bounds its band time from below.
# usage: tools/inst_mix.sh TAG CONFIG [LIB]
set -o pipefail
TAG=$1; CFG=$2; LIB=${3:+--lib $3}
export TMPDIR=/tmp
mkdir -p gpurun_out/imix_$TAG
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS \
  SQ_INSTS_VMEM SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/imix_$TAG/p1 -o run -- python3 bench.py \
  --config $CFG --no-cpu-baseline --no-random-leg --steps 6 --warmup 2 --timed-steps 2 $LIB \
  > gpurun_out/imix_$TAG/p1.log 2>&1 || { echo "inst-mix pass failed"; tail -5 gpurun_out/imix_$TAG/p1.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/imix_$TAG | tee gpurun_out/imix_$TAG/summary.txt | grep -A9 "stack"
