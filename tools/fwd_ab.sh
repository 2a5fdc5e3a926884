#!/bin/bash
# forward A/B: pipelined vs plain band kernel, and workgroup-geometry variants
export TMPDIR=/tmp
mkdir -p gpurun_out/fab
run() {  # tag
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fab/$1 -o run -- python3 tools/blockbench.py --reps 20 --what fwd > gpurun_out/fab/$1.log 2>&1 || { echo fail $1; tail gpurun_out/fab/$1.log; exit 1; }
  echo "== $1"; python3 tools/kstats.py gpurun_out/fab/$1/run_kernel_stats.csv 1
}
ASR_FWD_NOPIPE=1 run nopipe || exit 1
for v in 1 0 2; do ASR_FWD_VARIANT=$v run pipe_v$v || exit 1; done
