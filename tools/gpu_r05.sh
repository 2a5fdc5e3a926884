#!/bin/bash
# round-5 GPU call: the GPU suite + smoke on the in-tree build (TESTS=0 skips them),
# then whole-step A/B arms (tools/netab.sh, CONFIG/ARMS) and band stamps of
# trace builds (TRACES="tr0 tr3": build_abl_<name>.so).  Stops at the first
# step that crashed, hung or timed out.  usage: TAG=r05x [TESTS=1] [CONFIG=c2]
# [ARMS="cur t3 cur t3"] [TRACES=""] bash tools/gpu_r05.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05x}
crashed() { case $1 in 124|134|137|139) return 0;; esac; [ $1 -gt 128 ]; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -rfEs \
    > gpurun_out/test_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/test_$TAG.log
  [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)" gpurun_out/test_$TAG.log | head -20
  crashed $rc && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?
  tail -1 gpurun_out/smoke_$TAG.log
  crashed $rc && exit $rc
fi
if [ -n "$ARMS" ]; then
  timeout -k 10 900 bash tools/netab.sh ${CONFIG:-c2} "$ARMS" > gpurun_out/netab_$TAG.txt 2>&1; rc=$?
  cat gpurun_out/netab_$TAG.txt
  crashed $rc && exit $rc
fi
for t in $TRACES; do
  timeout -k 10 300 python tools/stacktrace.py build_abl_$t.so > gpurun_out/trace_${TAG}_$t.txt 2>&1; rc=$?
  echo "trace $t rc=$rc"; head -3 gpurun_out/trace_${TAG}_$t.txt
  crashed $rc && exit $rc
done
exit 0
