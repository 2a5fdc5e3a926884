#!/bin/bash
# Development round trip: GPU parity suite (or a subset), then short bench
# lines for the given configs.  usage: tools/gpu_dev.sh TAG "pytest args" cfg...
set -o pipefail
TAG=$1; PYARGS=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread $PYARGS > gpurun_out/test_$TAG.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/test_$TAG.log; exit 1; }
tail -1 gpurun_out/test_$TAG.log
for cfg in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo BENCH $cfg FAILED; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$cfg.json
done
