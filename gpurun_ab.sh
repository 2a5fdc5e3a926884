set -o pipefail
mkdir -p gpurun_out
bash tools/round_evidence.sh r02q || exit 1
export TMPDIR=/tmp
for cfg in c5 c3 c3_64; do
  timeout -k 10 400 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_r02q_$cfg.json 2> gpurun_out/bench_r02q_$cfg.err || { echo "bench $cfg failed"; tail -5 gpurun_out/bench_r02q_$cfg.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_r02q_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02q_c5 -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline > gpurun_out/prof_r02q_c5.log 2>&1 || { echo PROF c5 FAILED; exit 1; }
python3 tools/kstats.py gpurun_out/prof_r02q_c5/run_kernel_stats.csv 8
