#!/bin/bash
# Round-4 backward experiments: GPU tests of the stacked C=64 path on the in-tree
# build, then whole-step A/Bs of libasr builds (tools/netab.sh).
# usage: tools/gpu_r04d.sh TAG "ARMS"   (build_abl_<arm>.so built beforehand; "cur" = in-tree)
set -o pipefail
TAG=$1
ARMS=${2:-"head cur head cur head cur"}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stack64.py tests/test_gpu_headline.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/test_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/test_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|ERROR|Error" gpurun_out/test_$TAG.log | head -20; exit $rc; }
timeout -k 10 900 bash tools/netab.sh c2 "$ARMS" > gpurun_out/netab_$TAG.txt 2>&1; rc=$?; cat gpurun_out/netab_$TAG.txt; exit $rc
