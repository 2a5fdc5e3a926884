set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/test_r02r.log 2>&1 || { echo TESTS FAILED; grep -B5 -A30 "Error\|FAILED\|assert" gpurun_out/test_r02r.log | head -60; exit 1; }
tail -1 gpurun_out/test_r02r.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02r.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke_r02r.log; exit 1; }
tail -1 gpurun_out/smoke_r02r.log
timeout -k 10 400 python3 bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_r02r_c5.json 2> gpurun_out/bench_r02r_c5.err || { echo "bench c5 failed"; tail -5 gpurun_out/bench_r02r_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r02r_c5.json')); print('c5', d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r02r.json 2> gpurun_out/bench_r02r.err || { echo "bench c2 failed"; tail -5 gpurun_out/bench_r02r.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r02r.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash tools/netab.sh c2 "cur d4 d16 cur d4 d16" || exit 1
