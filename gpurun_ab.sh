set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_rk2.py tests/test_gpu_fullsize.py > gpurun_out/t3.log 2>&1; rc=$?
tail -1 gpurun_out/t3.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED\|assert" gpurun_out/t3.log | head -60; exit 1; }
timeout -k 10 200 python3 tools/blktrace.py build_abl_tr.so > gpurun_out/blktrace.txt 2>&1; tail -7 gpurun_out/blktrace.txt
AB_REPS=30 bash tools/ab.sh "${AB_LIST:-cur head cur head}" --what ${AB_WHAT:-bwd} 2>&1 | grep -v reduce_slabs
