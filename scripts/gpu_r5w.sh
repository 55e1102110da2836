#!/bin/bash
# CaffeNet step trace after the spill / scratch fixes
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cn6 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_cn6.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_cn6.log; exit 5; }
f=$(ls gpurun_out/prof_cn6/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_cn6/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_cn6_summary.txt && head -28 gpurun_out/prof_cn6_summary.txt
rm -rf gpurun_out/prof_cn6
