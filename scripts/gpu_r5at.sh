#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/plrn_probe.py 32768,49152,65536,98304 4,6,12,8,16,32 > gpurun_out/at_plrn.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/at_plrn.txt | grep -v "n/a" | tail -50
exit $rc
