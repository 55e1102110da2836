#!/bin/bash
# GoogLeNet b128 step trace: per-kernel summary and the stream timeline (critical path)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gn5 -o run --output-format csv -- python3 bench.py --model googlenet --steps 12 --warmup 4 --streams ${GN_STREAMS:-3} > gpurun_out/prof_gn5.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_gn5.log; exit 5; }
f=$(ls gpurun_out/prof_gn5/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_gn5/run_kernel_trace.csv)
head -1 "$f" | cut -c1-400
python3 scripts/prof_summary.py "$f" > gpurun_out/prof_gn5_summary.txt && head -32 gpurun_out/prof_gn5_summary.txt
python3 scripts/stream_timeline.py "$f" --top 30 > gpurun_out/gn5_timeline.txt; cat gpurun_out/gn5_timeline.txt
rm -rf gpurun_out/prof_gn5
