#!/bin/bash
# kernel-time of ablation builds (development)
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for v in ${ABL_LIST:-0 1 2 3}; do
  if [ $v = 0 ]; then unset ASR_LIB_OVERRIDE; else export ASR_LIB_OVERRIDE=$PWD/build_abl$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/v$v -o run -- python3 tools/blockbench.py --reps 20 --what "$@" > gpurun_out/abl/v$v.log 2>&1 || { echo fail $v; tail gpurun_out/abl/v$v.log; exit 1; }
  echo "== variant $v"; python3 tools/kstats.py gpurun_out/abl/v$v/run_kernel_stats.csv 3
done
