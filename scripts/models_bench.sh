#!/bin/bash
# 1-GPU bench of the zoo models at their defaults (one JSON line each -> gpurun_out/models_bench.jsonl).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/models_bench.jsonl
for spec in "caffenet --steps 20 --warmup 5" "alexnet --steps 20 --warmup 5" "googlenet --steps 20 --warmup 5" \
            "vgg16 --steps 10 --warmup 3" "vgg16 --steps 10 --warmup 3 --dtype fp8" "cifar10_quick --steps 200 --warmup 20" \
            "cifar10_full --steps 200 --warmup 20" "googlenet --steps 20 --warmup 5 --batch 256"; do
  timeout -k 10 300 python bench.py --model $spec >> gpurun_out/models_bench.jsonl 2> gpurun_out/models_bench.err || { echo "bench $spec failed"; tail -20 gpurun_out/models_bench.err; exit 1; }
  tail -1 gpurun_out/models_bench.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], d['config'].get('global_batch'), flush=True)"
done
