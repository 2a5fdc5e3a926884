#!/bin/bash
# development: rocprofv3 kernel times of blockbench for each build_abl_<name>.so (in-tree lib = "cur")
# usage: tools/ab.sh "name1 name2 ..." [blockbench args]
export TMPDIR=/tmp
LIST=$1; shift
mkdir -p gpurun_out/ab
for v in $LIST; do
  if [ $v = cur ]; then LIBARG=""; else LIBARG="--lib $PWD/build_abl_$v.so"; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$v -o run -- python3 ${AB_SCRIPT:-tools/blockbench.py} --reps ${AB_REPS:-20} $LIBARG "$@" > gpurun_out/ab/$v.log 2>&1 || { echo fail $v; tail gpurun_out/ab/$v.log; exit 1; }
  echo "== $v"; python3 tools/kstats.py gpurun_out/ab/$v/run_kernel_stats.csv 2 | tail -2
done
