#!/bin/bash
# Copy one GPU call's summaries from gpurun_out/ (scratch) into profiles/
# (tracked).  usage: tools/save_evidence.sh TAG
TAG=$1
cd "$(dirname "$0")/.."
mkdir -p profiles
[ -s gpurun_out/bench_$TAG.json ] && cp gpurun_out/bench_$TAG.json profiles/${TAG}_c2_bench.json
for f in gpurun_out/bench_${TAG}_*.json; do
  [ -s "$f" ] || continue; b=$(basename "$f" .json); cp "$f" profiles/${TAG}_${b#bench_${TAG}_}_bench.json
done
for d in gpurun_out/prof_${TAG}_*; do
  [ -d "$d" ] || continue
  cfg=${d##*_}
  cp $d/run_kernel_stats.csv profiles/${TAG}_${cfg}_kernel_stats.csv
  python3 tools/kstats.py $d/run_kernel_stats.csv 20 > profiles/${TAG}_${cfg}_kernel_stats.txt
  python3 tools/step_breakdown.py $d/run_kernel_trace.csv > profiles/${TAG}_${cfg}_step_breakdown.txt 2>/dev/null || true
done
[ -f gpurun_out/test_$TAG.log ] && tail -3 gpurun_out/test_$TAG.log > profiles/${TAG}_gpu_tests.txt
for d in gpurun_out/traffic_${TAG}*; do [ -d "$d" ] && cp $d/traffic_*.json profiles/ 2>/dev/null; done
for d in gpurun_out/pmc_${TAG}*; do [ -d "$d" ] && python3 tools/pmc_summary.py $d > profiles/$(basename $d).txt 2>&1; done
ls -la profiles | tail -20
