#!/bin/bash
# GoogLeNet b128 with the re-timed database: branch-stream count A/B (graph branches)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/gn_streams5.jsonl
for i in 1 2; do
  for s in 1 2 3 4 6; do
    timeout -k 10 300 python -u bench.py --model googlenet --streams $s >> gpurun_out/gn_streams5.jsonl 2> gpurun_out/gn_streams5.err || { tail -20 gpurun_out/gn_streams5.err; exit 5; }
    echo "googlenet streams=$s: $(tail -1 gpurun_out/gn_streams5.jsonl | cut -c45-75)"
  done
done
