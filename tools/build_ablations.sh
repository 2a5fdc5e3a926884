#!/bin/bash
# development: libasr variants with -DASR_ABLATE=k (see asr_block_mfma.hip)
cd "$(dirname "$0")/.."
S=differential_equations_resnet_amd/csrc
for k in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DASR_ABLATE=$k -o build_abl$k.so \
    $S/asr_theta.hip $S/asr_block_mfma.hip $S/asr_conv_f32.hip $S/asr_stem_head.hip $S/asr_api.hip &
done
wait
ls -la build_abl*.so
