#!/bin/bash
# GoogLeNet: packaged database vs the second isolated re-timing (after the spill fix), 3 pairs
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/gn_db2.jsonl
for i in 1 2 3; do
  for db in packaged retuned2; do
    if [ $db = packaged ]; then e=""; else e="SN_GEMM_TUNE_DB=gpurun_out/gemm_tuned_gn.json"; fi
    env $e timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/gn_db2.jsonl 2> gpurun_out/gn_db2.err || { tail -20 gpurun_out/gn_db2.err; exit 5; }
    echo "googlenet $db: $(tail -1 gpurun_out/gn_db2.jsonl | cut -c45-75)"
  done
done
