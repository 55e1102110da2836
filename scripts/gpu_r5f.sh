#!/bin/bash
# fp8 fidelity component A/B at lr 0.002 and 0.005
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for lr in 0.002 0.005; do
  timeout -k 10 900 python -u scripts/fp8_fidelity_ab.py $lr > gpurun_out/fp8_ab_$lr.txt 2>&1 || { tail -20 gpurun_out/fp8_ab_$lr.txt; exit 3; }
  grep -v amdgpu gpurun_out/fp8_ab_$lr.txt | tail -8
done
