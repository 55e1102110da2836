#!/bin/bash
# in-launch softmax-loss reduction: kernel + net + training tests, CaffeNet / GoogLeNet bench, CaffeNet step trace
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_net_gpu.py tests/test_training_gpu.py tests/test_bench_fidelity_gpu.py -m gpu > gpurun_out/aw_tests.log 2>&1 || { tail -40 gpurun_out/aw_tests.log; exit 3; }
tail -1 gpurun_out/aw_tests.log
: > gpurun_out/aw_bench.jsonl
for m in caffenet caffenet googlenet; do
  timeout -k 10 300 python -u bench.py --model $m >> gpurun_out/aw_bench.jsonl 2> gpurun_out/aw_bench.err || { tail -20 gpurun_out/aw_bench.err; exit 5; }
  echo "$m: $(tail -1 gpurun_out/aw_bench.jsonl | grep -o '"value": [0-9.]*')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cn10 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_cn10.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_cn10.log; exit 6; }
f=$(ls gpurun_out/prof_cn10/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_cn10/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_cn10_summary.txt && grep -n "xent\|softmax\|sum of" gpurun_out/prof_cn10_summary.txt | head -6
rm -rf gpurun_out/prof_cn10
