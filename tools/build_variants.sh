#!/bin/bash
# development: libasr variants for A/B timing.  usage: tools/build_variants.sh NAME "-DFLAG=.." [NAME "-D.."]...
# NAME=head builds the committed sources (git HEAD) instead of the working tree.
cd "$(dirname "$0")/.."
S=differential_equations_resnet_amd/csrc
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  src=$S
  if [ $name = head ]; then rm -rf /tmp/asr_head && mkdir -p /tmp/asr_head && git archive HEAD $S include | tar -x -C /tmp/asr_head && src=/tmp/asr_head/$S; fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared $flags -o build_abl_$name.so \
    $src/asr_theta.hip $src/asr_block_mfma.hip $src/asr_conv_f32.hip $src/asr_stem_head.hip $src/asr_api.hip $src/asr_dist.hip $src/asr_deep16.hip $src/asr_stages.hip &
done
wait
ls -la build_abl_*.so
