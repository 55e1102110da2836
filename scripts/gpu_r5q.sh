#!/bin/bash
# GoogLeNet: re-time every GEMM product in isolation into a copy of the database, then bench
# A/B (packaged database vs the re-timed copy), alternating
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
cp sparknet_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned_gn.json
timeout -k 10 900 python -u scripts/retune_isolated.py --model googlenet --out gpurun_out/gemm_tuned_gn.json > gpurun_out/retune_gn.txt 2>&1 || { tail -30 gpurun_out/retune_gn.txt; exit 4; }
tail -3 gpurun_out/retune_gn.txt
: > gpurun_out/retune_gn_ab.jsonl
for i in 1 2; do
  for db in packaged retuned; do
    if [ $db = packaged ]; then e=""; else e="SN_GEMM_TUNE_DB=gpurun_out/gemm_tuned_gn.json"; fi
    env $e timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/retune_gn_ab.jsonl 2> gpurun_out/retune_gn_ab.err || { tail -20 gpurun_out/retune_gn_ab.err; exit 5; }
    echo "googlenet $db: $(tail -1 gpurun_out/retune_gn_ab.jsonl | cut -c1-70)"
  done
done
cp sparknet_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned_cn.json
timeout -k 10 500 python -u scripts/retune_isolated.py --model caffenet --out gpurun_out/gemm_tuned_cn.json > gpurun_out/retune_cn.txt 2>&1 || { tail -30 gpurun_out/retune_cn.txt; exit 4; }
tail -1 gpurun_out/retune_cn.txt
: > gpurun_out/retune_cn_ab.jsonl
for i in 1 2; do
  for db in packaged retuned; do
    if [ $db = packaged ]; then e=""; else e="SN_GEMM_TUNE_DB=gpurun_out/gemm_tuned_cn.json"; fi
    env $e timeout -k 10 300 python -u bench.py >> gpurun_out/retune_cn_ab.jsonl 2> gpurun_out/retune_cn_ab.err || { tail -20 gpurun_out/retune_cn_ab.err; exit 5; }
    echo "caffenet $db: $(tail -1 gpurun_out/retune_cn_ab.jsonl | cut -c70-130)"
  done
done
