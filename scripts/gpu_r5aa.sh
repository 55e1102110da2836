#!/bin/bash
# final round-5 traces: GoogLeNet b128 (3 streams) with the stream timeline, VGG-16 b2048 bf16 and fp8
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
GN_STREAMS=3 bash scripts/gpu_r5p.sh > gpurun_out/gn_final.txt 2>&1 || { tail -5 gpurun_out/gn_final.txt; exit 5; }
grep -E "sum of kernel|iteration wall|in flight" gpurun_out/gn_final.txt
for dt in bf16 fp8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vgg_$dt -o run --output-format csv -- python3 bench.py --model vgg16 --dtype $dt --steps 3 --warmup 2 > gpurun_out/prof_vgg_$dt.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_vgg_$dt.log; exit 5; }
  f=$(ls gpurun_out/prof_vgg_$dt/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_vgg_$dt/run_kernel_trace.csv)
  python3 scripts/prof_summary.py "$f" > gpurun_out/prof_vgg_${dt}_summary.txt && tail -1 gpurun_out/prof_vgg_${dt}_summary.txt
  rm -rf gpurun_out/prof_vgg_$dt
done
