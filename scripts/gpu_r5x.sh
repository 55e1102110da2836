#!/bin/bash
# CaffeNet: only the memory-bound fused InnerProduct updates on the side stream (beside the
# compute-bound conv backward) vs inline, after the spill fix
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/fcs_ab.jsonl
for i in 1 2; do
  for cfg in "base" "SN_WGRAD_STREAM=1 SN_WGRAD_KINDS=fcsgd" "SN_WGRAD_STREAM=1 SN_WGRAD_KINDS=fc,fcsgd"; do
    if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
    env $e timeout -k 10 300 python -u bench.py >> gpurun_out/fcs_ab.jsonl 2> gpurun_out/fcs_ab.err || { tail -20 gpurun_out/fcs_ab.err; exit 5; }
    echo "$cfg: $(tail -1 gpurun_out/fcs_ab.jsonl | cut -c70-130)"
  done
done
