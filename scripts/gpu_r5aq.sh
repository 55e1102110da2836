#!/bin/bash
# 64-row tiles (21 / 22) for M not a multiple of 128 (e.g. 192): isolated re-time restricted to those tiles,
# then bench A/B (packaged database vs re-timed copy), CaffeNet and GoogLeNet, alternating
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for m in caffenet googlenet; do
  cp sparknet_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned_thin_$m.json
  timeout -k 10 900 python -u scripts/retune_isolated.py --model $m --tiles 21,22 --out gpurun_out/gemm_tuned_thin_$m.json > gpurun_out/retune_thin_$m.txt 2>&1 || { tail -30 gpurun_out/retune_thin_$m.txt; exit 4; }
  grep -- "->" gpurun_out/retune_thin_$m.txt | awk '$6 != $9' | head -30
  tail -1 gpurun_out/retune_thin_$m.txt
done
: > gpurun_out/thin_ab.jsonl
for i in 1 2; do
  for m in caffenet googlenet; do
    for db in packaged retuned; do
      if [ $db = packaged ]; then e=""; else e="SN_GEMM_TUNE_DB=gpurun_out/gemm_tuned_thin_$m.json"; fi
      env $e timeout -k 10 300 python -u bench.py --model $m >> gpurun_out/thin_ab.jsonl 2> gpurun_out/thin_ab.err || { tail -20 gpurun_out/thin_ab.err; exit 5; }
      echo "$m $db: $(tail -1 gpurun_out/thin_ab.jsonl | grep -o '"value": [0-9.]*')"
    done
  done
done
