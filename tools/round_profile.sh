#!/bin/bash
# Round evidence: default bench line, rocprofv3 kernel stats of the same
# command, PMC HBM traffic of one block.  usage: tools/round_profile.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 14
TRAFFIC_BLOCKS=30 bash tools/traffic.sh $TAG c2 --reps 3 --stack 30
