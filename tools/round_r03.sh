#!/bin/bash
# Round-3 evidence in one GPU call: the default bench line, rocprofv3 kernel
# stats + per-step breakdown of the same command, the eval / RK2 / C3 / C1
# bench lines, PMC HBM traffic and counters of the stacked C=64 kernels.
# Stops at the first failing step.  usage: tools/round_r03.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv 14
python3 tools/step_breakdown.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/prof_$TAG/step_breakdown.txt && cat gpurun_out/prof_$TAG/step_breakdown.txt
for cfg in c2_eval c5 c3 c1; do
  timeout -k 10 600 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "BENCH $cfg FAILED"; tail -5 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
TRAFFIC_BLOCKS=30 bash tools/traffic.sh $TAG c2 --reps 3 --stack 30 || exit 1
bash tools/pmc.sh $TAG --reps 3 --stack 30 || exit 1
