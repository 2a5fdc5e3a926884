#!/bin/bash
# Round-6 evidence in two GPU calls (each under gpurun's 20-minute limit).
# Part a: GPU suite, smoke, the default bench line, rocprofv3 kernel stats +
# per-step breakdowns (C2, he32_bf16, C3), the full-depth parity log, the r05k
# reproduction.  Part b: the other configs' bench lines, one PMC clock pass,
# PMC HBM traffic and counters of the stacked C=64 kernels.  Stops at the
# first failing step.  usage: tools/round_r06.sh TAG a|b
set -o pipefail
TAG=$1
PART=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$PART" = a ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -rfEs > gpurun_out/test_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/test_$TAG.log; [ $rc -le 1 ] || exit $rc
grep -E "FAILED|ERROR" gpurun_out/test_$TAG.log | head -10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_${TAG}_c2.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_${TAG}_c2.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_${TAG}_c2/run_kernel_stats.csv 14
python3 tools/step_breakdown.py gpurun_out/prof_${TAG}_c2/run_kernel_trace.csv > gpurun_out/prof_${TAG}_c2/step_breakdown.txt && cat gpurun_out/prof_${TAG}_c2/step_breakdown.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_he32bf16 -o run --output-format csv -- python3 bench.py --config he32_bf16 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_${TAG}_he32bf16.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_${TAG}_he32bf16.log; exit 1; }
python3 tools/step_breakdown.py gpurun_out/prof_${TAG}_he32bf16/run_kernel_trace.csv > gpurun_out/prof_${TAG}_he32bf16/step_breakdown.txt && head -12 gpurun_out/prof_${TAG}_he32bf16/step_breakdown.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_${TAG}_c3.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_${TAG}_c3.log; exit 1; }
python3 tools/step_breakdown.py gpurun_out/prof_${TAG}_c3/run_kernel_trace.csv > gpurun_out/prof_${TAG}_c3/step_breakdown.txt && head -8 gpurun_out/prof_${TAG}_c3/step_breakdown.txt
timeout -k 10 300 python -u -m pytest -q -s --timeout 250 --timeout-method thread tests/test_gpu_depth.py -p no:cacheprovider > gpurun_out/depth_$TAG.log 2>&1 || { echo DEPTH FAILED; tail -20 gpurun_out/depth_$TAG.log; exit 1; }
grep -E "^C[235]|balanced" gpurun_out/depth_$TAG.log
timeout -k 10 200 python tools/r05k_dead_channel.py > gpurun_out/r05k_$TAG.txt 2>&1 || { echo R05K FAILED; tail -5 gpurun_out/r05k_$TAG.txt; exit 1; }
cat gpurun_out/r05k_$TAG.txt
fi
if [ "$PART" = b ]; then
timeout -k 10 200 python tools/r05k_dead_channel.py > gpurun_out/r05k_${TAG}b.txt 2>&1 || { echo R05K FAILED; tail -5 gpurun_out/r05k_${TAG}b.txt; exit 1; }
for cfg in he32_bf16 he32 c2_eval c5 c3 c1 c2_f32 v6 v7_predict; do
  timeout -k 10 600 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "BENCH $cfg FAILED"; tail -5 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$cfg.json')); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['frac'], {k: v.get('avg_us') for k, v in r.get('kernels', {}).items()})"
done
bash tools/clock_pass.sh $TAG c2 || exit 1
TRAFFIC_BLOCKS=30 bash tools/traffic.sh $TAG c2 --reps 3 --stack 30 || exit 1
bash tools/pmc.sh $TAG --reps 3 --stack 30 || exit 1
fi
