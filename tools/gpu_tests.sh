set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/test_api1.log 2>&1; rc=$?
tail -40 gpurun_out/test_api1.log
exit $rc
