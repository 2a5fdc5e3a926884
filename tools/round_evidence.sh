#!/bin/bash
# Full round evidence on one GPU box: parity suite, default bench line,
# rocprofv3 kernel stats of the same command, PMC HBM traffic of one block.
# usage: tools/round_evidence.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/test_$TAG.log; exit 1; }
tail -1 gpurun_out/test_$TAG.log
bash tools/round_profile.sh $TAG
