#!/bin/bash
# GoogLeNet: dependency-free backward nodes (aux loss heads) on the least recently used branch stream (SN_BRANCH_DEPFREE) A/B + branch-stream tests
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
SN_BRANCH_DEPFREE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "branch or stream or googlenet or GoogLeNet" > gpurun_out/ax_tests.log 2>&1 || { tail -40 gpurun_out/ax_tests.log; exit 3; }
tail -1 gpurun_out/ax_tests.log
: > gpurun_out/ax_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    SN_BRANCH_DEPFREE=$v timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/ax_ab.jsonl 2> gpurun_out/ax_ab.err || { tail -20 gpurun_out/ax_ab.err; exit 5; }
    echo "googlenet depfree=$v: $(tail -1 gpurun_out/ax_ab.jsonl | grep -o '"value": [0-9.]*')"
  done
done
