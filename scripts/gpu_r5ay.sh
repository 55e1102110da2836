#!/bin/bash
# GoogLeNet with dependency-free nodes on LRU streams: 3 vs 4 branch streams
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/ay_ab.jsonl
for i in 1 2; do
  for n in 3 4 2; do
    timeout -k 10 300 python -u bench.py --model googlenet --streams $n >> gpurun_out/ay_ab.jsonl 2> gpurun_out/ay_ab.err || { tail -20 gpurun_out/ay_ab.err; exit 5; }
    echo "googlenet streams=$n: $(tail -1 gpurun_out/ay_ab.jsonl | grep -o '"value": [0-9.]*')"
  done
done
