#!/bin/bash
# VGG-16 b2048 bf16 step trace (regression hunt)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vgg5 -o run --output-format csv -- python3 bench.py --model vgg16 --steps 3 --warmup 2 > gpurun_out/prof_vgg5.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_vgg5.log; exit 5; }
f=$(ls gpurun_out/prof_vgg5/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_vgg5/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_vgg5_summary.txt && head -30 gpurun_out/prof_vgg5_summary.txt
rm -rf gpurun_out/prof_vgg5
