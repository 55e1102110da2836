#!/bin/bash
# bench window length: the same code at 50 / 200 / 400 timed steps (one host-latency step amortised)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/bd.jsonl
for m in caffenet googlenet; do
  for k in 50 200 400 50 200; do
    timeout -k 10 300 python -u bench.py --model $m --steps $k >> gpurun_out/bd.jsonl 2> gpurun_out/bd.err || { tail -20 gpurun_out/bd.err; exit 5; }
    echo "$m steps=$k: $(tail -1 gpurun_out/bd.jsonl | grep -o '"value": [0-9.]*')"
  done
done
