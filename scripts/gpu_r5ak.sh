#!/bin/bash
# GoogLeNet: every iteration's idle time under the kernel trace (is the 486 us gap per step?)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_gn8 -o run --output-format csv -- python3 bench.py --model googlenet --steps 12 --warmup 4 > gpurun_out/prof_gn8.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_gn8.log; exit 5; }
f=$(ls gpurun_out/prof_gn8/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_gn8/run_kernel_trace.csv)
python3 scripts/stream_timeline.py "$f" --iters --top 5 > gpurun_out/prof_gn8_timeline.txt; head -40 gpurun_out/prof_gn8_timeline.txt
tail -2 gpurun_out/prof_gn8.log
rm -rf gpurun_out/prof_gn8
