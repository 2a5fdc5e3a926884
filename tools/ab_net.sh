#!/bin/bash
# development: rocprofv3 kernel stats of a short bench.py run for each build
# usage: tools/ab_net.sh "name1 name2 ..." NTOP
export TMPDIR=/tmp
mkdir -p gpurun_out/abn
for v in $1; do
  if [ $v = cur ]; then unset ASR_LIB_OVERRIDE; else export ASR_LIB_OVERRIDE=$PWD/build_abl_$v.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abn/$v -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --block-reps 2 > gpurun_out/abn/$v.log 2>&1 || { echo fail $v; tail gpurun_out/abn/$v.log; exit 1; }
  echo "== $v"; python3 tools/kstats.py gpurun_out/abn/$v/run_kernel_stats.csv ${2:-12} | tail -n +2
done
