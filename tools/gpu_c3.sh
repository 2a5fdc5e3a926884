#!/bin/bash
# C3 (fused C=16 stack) evidence: step-stamps of the fused backward (trace build) + the c3 bench line.
# usage: tools/gpu_c3.sh TAG [TRACE_BUILD]
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$2" ]; then timeout -k 10 300 python3 tools/tracebench.py build_abl_$2.so > gpurun_out/c3trace_$TAG.txt 2>&1 || { echo TRACE FAILED; tail -20 gpurun_out/c3trace_$TAG.txt; exit 1; }; tail -6 gpurun_out/c3trace_$TAG.txt; fi
timeout -k 10 600 python3 bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || { echo "BENCH c3 FAILED"; tail -20 gpurun_out/bench_${TAG}_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_c3.json')); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], r['frac'], {k: (v.get('avg_us'), v.get('frac')) for k, v in r['kernels'].items()})"
