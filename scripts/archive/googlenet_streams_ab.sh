#!/bin/bash
# GoogLeNet batch 128: branch-stream count A/B (engine.BranchStreams), interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/gn_streams.jsonl
for st in 4 6 8 3 4 6 8; do
  timeout -k 10 300 python bench.py --model googlenet --steps 30 --warmup 5 --streams $st >> gpurun_out/gn_streams.jsonl 2> gpurun_out/gn_streams.err || { echo "bench streams $st failed"; tail -20 gpurun_out/gn_streams.err; exit 1; }
  tail -1 gpurun_out/gn_streams.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams $st', d['value'], d['ms_per_step'], flush=True)"
done
