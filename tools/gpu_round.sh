#!/bin/bash
# One GPU call of round evidence: the GPU parity suite (no -x: every failure
# is listed), smoke(), the default bench line, rocprofv3 kernel stats of the
# bench command, PMC HBM traffic and counters of one block.  Stops at the
# first step that crashes or times out (exit status > 1).
# usage: tools/gpu_round.sh TAG [steps...]   steps: tests smoke bench prof traffic pmc
set -o pipefail
TAG=$1; shift
STEPS=${*:-tests smoke bench prof traffic pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "== $what rc=$rc"; if [ $rc -gt 1 ]; then echo "stopping after $what (rc $rc)"; exit $rc; fi; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -rfEs > gpurun_out/test_$TAG.log 2>&1
      rc=$?; tail -40 gpurun_out/test_$TAG.log; ok $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
      rc=$?; tail -3 gpurun_out/smoke_$TAG.log; ok $rc smoke ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
      rc=$?; cat gpurun_out/bench_$TAG.json; tail -8 gpurun_out/bench_$TAG.err; ok $rc bench ;;
    bench_*)
      cfg=${s#bench_}
      timeout -k 10 600 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err
      rc=$?; cat gpurun_out/bench_${TAG}_$cfg.json; tail -5 gpurun_out/bench_${TAG}_$cfg.err; ok $rc $s ;;
    prof|prof_*)
      cfg=c2; [ $s != prof ] && cfg=${s#prof_}
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_${TAG}_$cfg.log 2>&1
      rc=$?; python3 tools/kstats.py gpurun_out/prof_${TAG}_$cfg/run_kernel_stats.csv 14; tail -2 gpurun_out/prof_${TAG}_$cfg.log; ok $rc $s ;;
    traffic)
      bash tools/traffic.sh $TAG c2 --reps 10; ok $? traffic ;;
    traffic_c3)
      bash tools/traffic.sh ${TAG}_c3 c3 --reps 10 --C 16 --N 1024; ok $? traffic_c3 ;;
    pmc)
      bash tools/pmc.sh $TAG --reps 10; ok $? pmc ;;
  esac
done
