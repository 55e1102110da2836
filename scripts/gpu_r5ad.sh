#!/bin/bash
# fp8 fidelity at the production learning rate (lr 0.005) and 0.003, after the round-5 fixes
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for lr in 0.005 0.003; do
  for b in 1 0; do
    SN_FP8_FID_LR=$lr SN_FP8_WGRAD_BIAS=$b timeout -k 10 600 python -u -m pytest -q -s --timeout 500 --timeout-method thread tests/test_fp8_fidelity_gpu.py -m gpu > gpurun_out/fid_lr${lr}_b$b.log 2>&1; rc=$?
    echo "lr $lr bias $b rc=$rc: $(grep -E "chaos floor" gpurun_out/fid_lr${lr}_b$b.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
