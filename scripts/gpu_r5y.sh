#!/bin/bash
# CaffeNet with the fused FC updates on a side stream: timeline (where the 20 % goes)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export SN_WGRAD_STREAM=1 SN_WGRAD_KINDS=fcsgd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fcs -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 > gpurun_out/prof_fcs.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_fcs.log; exit 5; }
f=$(ls gpurun_out/prof_fcs/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_fcs/run_kernel_trace.csv)
python3 scripts/stream_timeline.py "$f" --top 20 > gpurun_out/fcs_timeline.txt; cat gpurun_out/fcs_timeline.txt
python3 scripts/prof_summary.py "$f" > gpurun_out/fcs_summary.txt; head -12 gpurun_out/fcs_summary.txt
rm -rf gpurun_out/prof_fcs
