#!/bin/bash
# development: whole-step A/B of libasr builds (build_abl_<name>.so) on one box:
# each arm's library replaces the in-tree libasr.so of this (scratch) copy in
# turn, then one short bench.py run.  usage: tools/netab.sh CONFIG "a b a b"
cfg=$1; arms=$2
mkdir -p gpurun_out/netab
lib=differential_equations_resnet_amd/libasr.so
for v in $arms; do
  cp build_abl_$v.so $lib
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 30 --warmup 5 --block-reps 5 \
    > gpurun_out/netab/$v.json 2> gpurun_out/netab/$v.err || { echo "fail $v"; tail -5 gpurun_out/netab/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/netab/$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
