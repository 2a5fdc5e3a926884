#!/bin/bash
# the full GPU suite + smoke on the in-tree build, then a whole-step A/B against a
# previous build (build_abl_head.so).  usage: tools/gpu_verify.sh TAG ["ARMS"]
set -o pipefail
TAG=$1
ARMS=${2:-"head cur head cur head cur"}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -rfEs > gpurun_out/test_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/test_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|ERROR" gpurun_out/test_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 bash tools/netab.sh c2 "$ARMS" > gpurun_out/netab_$TAG.txt 2>&1; rc=$?; cat gpurun_out/netab_$TAG.txt; exit $rc
