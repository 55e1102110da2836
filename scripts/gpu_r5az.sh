#!/bin/bash
# GoogLeNet: off-trunk branches (aux loss heads in forward) leave the main stream (SN_BRANCH_OFFTRUNK) A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
SN_BRANCH_OFFTRUNK=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_net_gpu.py -m gpu -k "branch or stream or googlenet or GoogLeNet" > gpurun_out/az_tests.log 2>&1 || { tail -40 gpurun_out/az_tests.log; exit 3; }
tail -1 gpurun_out/az_tests.log
: > gpurun_out/az_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    SN_BRANCH_OFFTRUNK=$v timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/az_ab.jsonl 2> gpurun_out/az_ab.err || { tail -20 gpurun_out/az_ab.err; exit 5; }
    echo "googlenet offtrunk=$v: $(tail -1 gpurun_out/az_ab.jsonl | grep -o '"value": [0-9.]*')"
  done
done
