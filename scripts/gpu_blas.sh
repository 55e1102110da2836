#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 python3 -u scripts/gemm_vs_blas.py > gpurun_out/gemm_vs_blas.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/gemm_vs_blas.txt; exit $rc
