#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/fv
for v in 0 1 2 3; do
  export ASR_FWD_VARIANT=$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fv/v$v -o run -- python3 tools/blockbench.py --reps 20 --what "$@" > gpurun_out/fv/v$v.log 2>&1 || { echo fail $v; tail gpurun_out/fv/v$v.log; exit 1; }
  echo "== variant $v"; python3 tools/kstats.py gpurun_out/fv/v$v/run_kernel_stats.csv 2
done
