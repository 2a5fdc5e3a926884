#!/bin/bash
# Round-4 check of the graceful hand-off: the stack64 and distributed GPU tests,
# the default bench line, the clock/MFMA-busy PMC pass.  usage: tools/gpu_r04a.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_stack64.py tests/test_gpu_distributed.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/test_$TAG.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/test_$TAG.log; exit 1; }
tail -3 gpurun_out/test_$TAG.log
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash tools/clock_pass.sh $TAG c2
