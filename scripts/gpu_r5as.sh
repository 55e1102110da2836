#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/plrn_check.py 256 sweep > gpurun_out/as_check2.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/as_check2.txt | tail -40
exit $rc
