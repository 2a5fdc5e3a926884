#!/bin/bash
# Development: block-kernel parity tests, then rocprofv3 kernel times of one
# block fwd+bwd at the C2 shape.  usage: tools/gpu_blk.sh TAG [pytest -k expr]
set -o pipefail
TAG=$1; K=${2:-"parity or rk2 or projection or dgrad"}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_rk2.py -k "$K" > gpurun_out/test_$TAG.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/test_$TAG.log; exit 1; }
tail -1 gpurun_out/test_$TAG.log
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/blk_$TAG -o run -- python3 tools/blockbench.py --reps 20 > gpurun_out/blk_$TAG.log 2>&1 || { echo PROF FAILED; tail gpurun_out/blk_$TAG.log; exit 1; }
python3 tools/kstats.py gpurun_out/blk_$TAG/run_kernel_stats.csv 4
