set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stack64.py > gpurun_out/t_st.log 2>&1; rc=$?
tail -3 gpurun_out/t_st.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED\|assert" gpurun_out/t_st.log | head -80; exit 1; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_fullsize.py tests/test_gpu_network.py tests/test_gpu_api.py > gpurun_out/t_fs.log 2>&1; rc=$?
tail -3 gpurun_out/t_fs.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED\|assert" gpurun_out/t_fs.log | head -80; exit 1; }
bash tools/netab.sh c2 "base fwd both base fwd both"
