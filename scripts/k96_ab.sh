#!/bin/bash
# Direct 48 -> 96-channel conv for CaffeNet conv1 (after the S2D fold) vs the implicit GEMM.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_quick.sh tests/test_kernels_gpu.py -k "conv3x3" || exit 1
for r in ${REPS:-1 2 3}; do
  for v in 1 0; do
    SN_CONV_DIRECT_K96=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('caffenet direct_k96=$v', d['value'], d['ms_per_step'], d['config']['final_loss'], flush=True)" || exit 1
  done
done
