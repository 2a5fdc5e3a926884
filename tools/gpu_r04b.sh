#!/bin/bash
# Round-4 pair-local slabs + small batches: GPU tests, the same-process A/B (pair vs
# ASR_VARIANT_FULL_SLABS), the default bench line and the new configs.
# usage: tools/gpu_r04b.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_stack64.py tests/test_gpu_headline.py tests/test_gpu_distributed.py "tests/test_gpu_fullsize.py::test_v6_small_batch_and_batch1_predict" tests/test_gpu_kernels.py tests/test_gpu_api.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/test_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/test_$TAG.log; [ $rc -le 1 ] || exit $rc
grep -E "FAILED|ERROR" gpurun_out/test_$TAG.log | head -20
timeout -k 10 600 python3 tools/varab.py --config c2 --arms 0,256 --rounds 6 > gpurun_out/varab_$TAG.txt 2>&1 || { echo VARAB FAILED; tail -20 gpurun_out/varab_$TAG.txt; exit 1; }
cat gpurun_out/varab_$TAG.txt
for cfg in c2 v6 v7_predict c2_f32 v6_f32; do
  timeout -k 10 600 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err || { echo "BENCH $cfg FAILED"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$cfg.json')); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], d['vs_baseline'], r['frac'], {k: v.get('avg_us') for k, v in r['kernels'].items()}, r.get('mfma_frac_held_clock'), r.get('hbm_frac_at_mfma_ceiling'))"
done
