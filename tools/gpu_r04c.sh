#!/bin/bash
# Round-4 diagnostics of the pair-local build: band stamps of the C=64 stacks
# (trace build), PMC HBM traffic and counters of the stacks.
# usage: tools/gpu_r04c.sh TAG   (build_abl_tr.so built beforehand)
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/stacktrace.py build_abl_tr.so > gpurun_out/trace_$TAG.txt 2>&1 || { echo TRACE FAILED; tail -20 gpurun_out/trace_$TAG.txt; exit 1; }
head -60 gpurun_out/trace_$TAG.txt
TRAFFIC_BLOCKS=30 bash tools/traffic.sh $TAG c2 --reps 3 --stack 30 || exit 1
bash tools/pmc.sh $TAG --reps 3 --stack 30 || exit 1
