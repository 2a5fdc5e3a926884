#!/bin/bash
# tests + default bench line (no cpu baseline) + kernel stats.  usage: tools/gpu_quick.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/test_$TAG.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/test_$TAG.log; exit 1; }
tail -1 gpurun_out/test_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 8
