#!/bin/bash
# cifar10_quick learning regression: default / no thin re-tune / no autotune; fp8 fidelity setting sweep (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for v in "" "SN_GRAPH_RELEASE=1" "SN_GEMM_THIN_RETUNE=0" "SN_GEMM_AUTOTUNE=0"; do
  env $v SN_GEMM_TUNE_LOG=1 timeout -k 10 200 python -u -m pytest tests/test_training_gpu.py -x -q -rf --timeout 120 --timeout-method thread -s -k cifar10_quick > "gpurun_out/dbg_cifar_${v:-default}.log" 2>&1
  echo "== ${v:-default} rc=$?"; grep -E "passed|failed|AssertionError" "gpurun_out/dbg_cifar_${v:-default}.log" | head -3
done
LRS="0.002 0.001" bash scripts/gpu_fp8d.sh
