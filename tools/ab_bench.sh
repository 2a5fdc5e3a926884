#!/bin/bash
# development: whole-step A/B of library builds (bench.py images/s), alternating.
# usage: tools/ab_bench.sh "name1 name2 ..." [bench args]   (cur = in-tree lib)
LIST=$1; shift
for v in $LIST; do
  if [ $v = cur ]; then unset ASR_LIB_OVERRIDE; else export ASR_LIB_OVERRIDE=$PWD/build_abl_$v.so; fi
  r=$(timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 --block-reps 10 "$@" 2>/dev/null) || { echo "fail $v"; exit 1; }
  echo "$v $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_us_fwd"], r["avg_us_bwd"], r["avg_us"])')"
done
