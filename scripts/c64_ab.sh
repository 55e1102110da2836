#!/bin/bash
# Direct 64-channel 3x3 conv (8 / 4 waves) vs the implicit GEMM for VGG-16's conv1_2 products.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_quick.sh tests/test_kernels_gpu.py -k "conv3x3" || exit 1
SN_C64_WAVES=4 bash scripts/gpu_quick.sh tests/test_kernels_gpu.py -k "conv3x3" || exit 1
for r in 1 2; do
  for v in "SN_C64_WAVES=8" "SN_C64_WAVES=4" "SN_CONV_DIRECT_C64=0"; do
    env $v timeout -k 10 300 python bench.py --model vgg16 --steps 6 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('vgg16 $v', d['value'], d['ms_per_step'], d['config']['final_loss'], flush=True)" || exit 1
  done
done
