#!/bin/bash
# development: whole-step A/B of environment switches on the in-tree library (bench.py images/s), alternating.
# usage: tools/ab_env.sh "VAR=1 -" [bench args]   ("-" = no extra variable)
LIST=$1; shift
for v in $LIST; do
  if [ "$v" = "-" ]; then envs=(); else envs=("$v"); fi
  r=$(env "${envs[@]}" timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 --block-reps 10 "$@" 2>/dev/null) || { echo "fail $v"; exit 1; }
  echo "$v $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_us_fwd"], r["avg_us_bwd"], r["avg_us"])')"
done
