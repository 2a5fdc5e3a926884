set -o pipefail
mkdir -p gpurun_out
for v in cur fh; do
  cp build_abl_$v.so differential_equations_resnet_amd/libasr.so
  timeout -k 10 200 python3 -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_stack64.py tests/test_gpu_headline.py > gpurun_out/t_$v.log 2>&1 || { echo "$v FAILED"; tail -30 gpurun_out/t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_$v.log)"
done
bash tools/netab.sh c2 "cur fh cur fh" || exit 1
cp build_abl_cur.so differential_equations_resnet_amd/libasr.so
TRAFFIC_BLOCKS=30 bash tools/traffic.sh r02o c2 --reps 3 --stack 30 || exit 1
