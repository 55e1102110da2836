#!/bin/bash
# batched-load average pooling: pool tests, GoogLeNet bench x3, GoogLeNet step trace (avepool share)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "pool" > gpurun_out/ap_tests.log 2>&1 || { tail -40 gpurun_out/ap_tests.log; exit 3; }
tail -1 gpurun_out/ap_tests.log
: > gpurun_out/ap_bench.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/ap_bench.jsonl 2> gpurun_out/ap_bench.err || { tail -20 gpurun_out/ap_bench.err; exit 5; }
  echo "googlenet: $(tail -1 gpurun_out/ap_bench.jsonl | cut -c45-75)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gn7 -o run --output-format csv -- python3 bench.py --model googlenet --steps 10 --warmup 5 > gpurun_out/prof_gn7.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_gn7.log; exit 6; }
f=$(ls gpurun_out/prof_gn7/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_gn7/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_gn7_summary.txt && head -40 gpurun_out/prof_gn7_summary.txt
python3 scripts/stream_timeline.py "$f" > gpurun_out/prof_gn7_timeline.txt
rm -rf gpurun_out/prof_gn7
