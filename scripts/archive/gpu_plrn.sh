#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 180 python3 scripts/plrn_probe.py "20000,32768,48000" 4,8 > gpurun_out/plrn_probe2.txt 2>&1 || { cat gpurun_out/plrn_probe2.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/plrn_probe2.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "lrn or pool" --timeout 120 --timeout-method thread > gpurun_out/plrn_tests.log 2>&1 || { tail -20 gpurun_out/plrn_tests.log; exit 4; }
tail -2 gpurun_out/plrn_tests.log
for i in 1 2; do timeout -k 10 300 python -u bench.py 2>/dev/null | grep -o '"value": [0-9.]*'; done
