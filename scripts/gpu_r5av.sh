#!/bin/bash
# 16-byte flip_weights_multi: flip / conv tests, smoke(), CaffeNet bench x2 + step trace (flip time)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "flip or conv" > gpurun_out/av_tests.log 2>&1 || { tail -40 gpurun_out/av_tests.log; exit 3; }
tail -1 gpurun_out/av_tests.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids | tail -2
: > gpurun_out/av_bench.jsonl
for v in 1 0 1 0; do
  SN_FLIP_VEC=$v timeout -k 10 300 python -u bench.py >> gpurun_out/av_bench.jsonl 2> gpurun_out/av_bench.err || { tail -20 gpurun_out/av_bench.err; exit 5; }
  echo "caffenet flip_vec=$v: $(tail -1 gpurun_out/av_bench.jsonl | grep -o '"value": [0-9.]*')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cn9 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_cn9.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_cn9.log; exit 6; }
f=$(ls gpurun_out/prof_cn9/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_cn9/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_cn9_summary.txt && grep -n "flip\|sum of" gpurun_out/prof_cn9_summary.txt | head -4
rm -rf gpurun_out/prof_cn9
