#!/bin/bash
# CaffeNet / cifar10: isolated re-timing into a copy of the (GoogLeNet-updated) database, bench A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
cp sparknet_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned_cn.json
timeout -k 10 500 python -u scripts/retune_isolated.py --model caffenet --out gpurun_out/gemm_tuned_cn.json > gpurun_out/retune_cn.txt 2>&1 || { tail -30 gpurun_out/retune_cn.txt; exit 4; }
tail -2 gpurun_out/retune_cn.txt
for m in cifar10_quick cifar10_full; do
  timeout -k 10 300 python -u scripts/retune_isolated.py --model $m --out gpurun_out/gemm_tuned_cn.json > gpurun_out/retune_$m.txt 2>&1 || { tail -30 gpurun_out/retune_$m.txt; exit 4; }
  tail -1 gpurun_out/retune_$m.txt
done
: > gpurun_out/retune_cn_ab.jsonl
for i in 1 2; do
  for db in packaged retuned; do
    if [ $db = packaged ]; then e=""; else e="SN_GEMM_TUNE_DB=gpurun_out/gemm_tuned_cn.json"; fi
    env $e timeout -k 10 300 python -u bench.py >> gpurun_out/retune_cn_ab.jsonl 2> gpurun_out/retune_cn_ab.err || { tail -20 gpurun_out/retune_cn_ab.err; exit 5; }
    echo "caffenet $db: $(tail -1 gpurun_out/retune_cn_ab.jsonl | cut -c70-130)"
  done
done
