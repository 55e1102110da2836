#!/bin/bash
# new fused LRN/pool backward tile chooser: fused pool/LRN tests, correctness check at b256, CaffeNet bench x2 + step trace
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pool_lrn_gpu.py -m gpu > gpurun_out/au_tests.log 2>&1 || { tail -40 gpurun_out/au_tests.log; exit 3; }
tail -1 gpurun_out/au_tests.log
timeout -k 10 200 python -u scripts/plrn_check.py 256 2>&1 | grep -v amdgpu
: > gpurun_out/au_bench.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py >> gpurun_out/au_bench.jsonl 2> gpurun_out/au_bench.err || { tail -20 gpurun_out/au_bench.err; exit 5; }
  echo "caffenet: $(tail -1 gpurun_out/au_bench.jsonl | grep -o '"value": [0-9.]*')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cn8 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_cn8.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_cn8.log; exit 6; }
f=$(ls gpurun_out/prof_cn8/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_cn8/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_cn8_summary.txt && grep -n "lrn\|sum of" gpurun_out/prof_cn8_summary.txt | head
rm -rf gpurun_out/prof_cn8
