set -o pipefail
mkdir -p gpurun_out
bash tools/netab.sh c2 "cur d4 d16 cur d4 d16" || exit 1
