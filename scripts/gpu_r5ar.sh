#!/bin/bash
# fused LRN/pool backward tile sweep in isolation (after the sn_powneg change): LDS budgets x channel groups
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/plrn_probe.py 32768,49152,65536,98304 4,6,12,8,16,32 > gpurun_out/ar_plrn.txt 2>&1 || { tail -20 gpurun_out/ar_plrn.txt; exit 4; }
grep -v amdgpu.ids gpurun_out/ar_plrn.txt | grep -v "n/a" | sort -t: -k2 -n | head -80
