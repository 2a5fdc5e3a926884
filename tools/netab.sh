#!/bin/bash
# development: whole-step A/B of libasr builds (build_abl_<name>.so, "cur" = the
# in-tree libasr.so) on one box.  Each arm runs in its own process and loads its
# build through bench.py --lib; the in-tree library is never replaced.
# usage: tools/netab.sh CONFIG "a b a b"
cfg=$1; arms=$2
mkdir -p gpurun_out/netab
for v in $arms; do
  if [ $v = cur ]; then LIBARG=""; else LIBARG="--lib $PWD/build_abl_$v.so"; fi
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 30 --warmup 5 --block-reps 5 $LIBARG \
    > gpurun_out/netab/$v.json 2> gpurun_out/netab/$v.err || { echo "fail $v"; tail -5 gpurun_out/netab/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/netab/$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
