#!/bin/bash
# r6: baseline bench on this round's box + weight-gradient anatomy probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || exit 1
cat gpurun_out/r6a_bench.json
timeout -k 10 600 python -u scripts/wgrad_probe.py > gpurun_out/r6a_wgrad.txt 2>&1
echo "probe rc $?"
tail -40 gpurun_out/r6a_wgrad.txt
