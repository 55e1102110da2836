#!/bin/bash
# the fp8 fidelity test as committed (lr 0.002 and 0.005, cost-model tiles), twice
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest -q -s --timeout 500 --timeout-method thread tests/test_fp8_fidelity_gpu.py -m gpu > gpurun_out/fid_final_$i.log 2>&1; rc=$?
  grep -E "^lr|chaos floor|passed|failed" gpurun_out/fid_final_$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
