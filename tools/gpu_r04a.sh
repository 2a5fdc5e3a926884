#!/bin/bash
# Round-4 checks: the fp32 MFMA kernels and the graceful hand-off (GPU tests),
# the default bench line, C1, the clock/MFMA-busy PMC pass.  usage: tools/gpu_r04a.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_network.py tests/test_gpu_rk2.py "tests/test_gpu_fullsize.py::test_c1_fullsize_fp32_vs_reference_graph" -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/test_f32_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/test_f32_$TAG.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_stack64.py tests/test_gpu_distributed.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/test_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/test_$TAG.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 python3 bench.py --config c1 --no-cpu-baseline > gpurun_out/bench_${TAG}_c1.json 2> gpurun_out/bench_${TAG}_c1.err || { echo BENCH C1 FAILED; tail -20 gpurun_out/bench_${TAG}_c1.err; exit 1; }
cat gpurun_out/bench_${TAG}_c1.json
bash tools/clock_pass.sh $TAG c2
