#!/bin/bash
# A/B + band stamps of backward variants. usage: tools/gpu_r04n.sh TAG "ARMS" "TRACE_BUILDS"
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack64.py tests/test_gpu_headline.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/test_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/test_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|ERROR|Error" gpurun_out/test_$TAG.log | head -20; exit $rc; }
timeout -k 10 900 bash tools/netab.sh c2 "$2" > gpurun_out/netab_$TAG.txt 2>&1; rc=$?; cat gpurun_out/netab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
[ -n "$3" ] && bash tools/gpu_trace.sh $TAG "$3"
exit 0
