#!/bin/bash
# final-code step traces: GoogLeNet b128 and CaffeNet b256 (per-kernel sums, stream timeline)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gnf -o run --output-format csv -- python3 bench.py --model googlenet --steps 12 --warmup 4 > gpurun_out/prof_gnf.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_gnf.log; exit 5; }
f=$(ls gpurun_out/prof_gnf/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_gnf/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_gnf_summary.txt && head -32 gpurun_out/prof_gnf_summary.txt
python3 scripts/stream_timeline.py "$f" --iters --top 10 > gpurun_out/prof_gnf_timeline.txt; sed -n 1,30p gpurun_out/prof_gnf_timeline.txt | grep -v "^iter [0-2]:"
rm -rf gpurun_out/prof_gnf
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnf -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_cnf.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_cnf.log; exit 6; }
f=$(ls gpurun_out/prof_cnf/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_cnf/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_cnf_summary.txt && head -3 gpurun_out/prof_cnf_summary.txt && grep "sum of" gpurun_out/prof_cnf_summary.txt
rm -rf gpurun_out/prof_cnf
