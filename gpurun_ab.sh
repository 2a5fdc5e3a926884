set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stack64.py tests/test_gpu_rk2.py > gpurun_out/t_rk.log 2>&1; rc=$?
tail -2 gpurun_out/t_rk.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED\|assert" gpurun_out/t_rk.log | head -70; exit 1; }
bash tools/netab.sh c5 "nobs cur nobs cur" || exit 1
