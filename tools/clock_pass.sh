#!/bin/bash
# One PMC pass over the bench command (the network's own block kernels): held
# clock, MFMA busy and VALU per MFMA of the stack kernels -> clock_<config>.json
# usage: tools/clock_pass.sh TAG CONFIG
set -o pipefail
TAG=$1; CFG=$2
export TMPDIR=/tmp
mkdir -p gpurun_out/clock_$TAG
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace \
  --output-format csv -d gpurun_out/clock_$TAG/p1 -o run -- python3 bench.py --config $CFG --no-cpu-baseline \
  --no-random-leg --steps 10 --warmup 3 --timed-steps 2 > gpurun_out/clock_$TAG/p1.log 2>&1 \
  || { echo "clock pass failed"; tail -5 gpurun_out/clock_$TAG/p1.log; exit 1; }
python3 tools/clock.py gpurun_out/clock_$TAG $CFG gpurun_out/clock_$TAG/clock_$CFG.json $TAG
