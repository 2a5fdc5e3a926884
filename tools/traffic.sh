#!/bin/bash
# HBM traffic (PMC) of one Euler block fwd+bwd at the C2 shape: two separate
# counter passes (no tracing domains besides --kernel-trace).
# usage: tools/traffic.sh TAG CONFIG [blockbench args]
set -o pipefail
TAG=$1; CFG=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic_$TAG
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/traffic_$TAG/p$i -o run -- python3 tools/blockbench.py "$@" > gpurun_out/traffic_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/traffic_$TAG/p$i.log; exit 1; }
done
python3 tools/traffic.py gpurun_out/traffic_$TAG $CFG gpurun_out/traffic_$TAG/traffic_$CFG.json $TAG ${TRAFFIC_BLOCKS:-1}
