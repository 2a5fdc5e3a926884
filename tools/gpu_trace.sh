#!/bin/bash
# band stamps of the C=64 stacks for several trace builds (build_abl_<name>.so)
# usage: tools/gpu_trace.sh TAG "name1 name2 ..."
set -o pipefail
TAG=$1
mkdir -p gpurun_out
for v in $2; do
  timeout -k 10 200 python3 tools/stacktrace.py build_abl_$v.so > gpurun_out/trace_${TAG}_$v.txt 2>&1 || { echo "TRACE $v FAILED"; tail -20 gpurun_out/trace_${TAG}_$v.txt; exit 1; }
  echo "== $v"; head -3 gpurun_out/trace_${TAG}_$v.txt | tail -2
done
