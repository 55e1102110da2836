#!/bin/bash
# VGG-16 b2048 fp8: the colsum (exact bias gradient) and quant launches of one step
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v8 -o run --output-format csv -- python3 bench.py --model vgg16 --dtype fp8 --steps 3 --warmup 2 > gpurun_out/prof_v8.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_v8.log; exit 5; }
f=$(ls gpurun_out/prof_v8/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_v8/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_v8_all.txt; grep -B2 -A2 "colsum_pass1" gpurun_out/prof_v8_all.txt | grep grid | cut -c1-120 | head -60
rm -rf gpurun_out/prof_v8
