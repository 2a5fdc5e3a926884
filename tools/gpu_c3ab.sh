#!/bin/bash
# C3 A/B of libasr builds + step stamps of trace builds.  usage: tools/gpu_c3ab.sh TAG "ARMS" "TRACE_BUILDS"
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $3; do
  timeout -k 10 300 python3 tools/tracebench.py build_abl_$v.so > gpurun_out/c3trace_${TAG}_$v.txt 2>&1 || { echo "TRACE $v FAILED"; tail -20 gpurun_out/c3trace_${TAG}_$v.txt; exit 1; }
  echo "== $v"; tail -5 gpurun_out/c3trace_${TAG}_$v.txt
done
timeout -k 10 900 bash tools/netab.sh c3 "$2" > gpurun_out/c3ab_$TAG.txt 2>&1; rc=$?; cat gpurun_out/c3ab_$TAG.txt; exit $rc
