#!/bin/bash
# packed conv1 kernel: numerics, then CaffeNet bench A/B (packed vs 64-channel direct), then a step trace
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "packed or k96" --timeout 120 --timeout-method thread > gpurun_out/packed_tests.log 2>&1 || { tail -30 gpurun_out/packed_tests.log; exit 3; }
tail -3 gpurun_out/packed_tests.log
: > gpurun_out/packed_ab.jsonl
for v in 1 0 1 0; do
  SN_CONV_PACKED=$v timeout -k 10 300 python -u bench.py >> gpurun_out/packed_ab.jsonl 2> gpurun_out/packed_ab.err || { tail -20 gpurun_out/packed_ab.err; exit 4; }
  echo "packed=$v $(tail -1 gpurun_out/packed_ab.jsonl | cut -c1-120)"
done
rm -rf gpurun_out/prof_packed
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_packed -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/prof_packed.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_packed.log; exit 5; }
python3 scripts/prof_summary.py gpurun_out/prof_packed > gpurun_out/prof_packed_summary.txt 2>&1
head -30 gpurun_out/prof_packed_summary.txt
