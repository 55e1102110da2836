#!/bin/bash
# VGG-16 b2048 fp8: cost-model threshold A/B now that conv1_1 -> conv1_2 can hand over e4m3
# bytes from its epilogue (fused quantisation) — 1000 keeps conv1_2 / conv2_1-dgrad in bf16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/fp8_minwork.jsonl
for w in 500 1000 0 500 1000; do
  timeout -k 10 400 python bench.py --model vgg16 --steps 8 --warmup 3 --dtype fp8 --fp8-min-work $w >> gpurun_out/fp8_minwork.jsonl 2> gpurun_out/fp8_minwork.err || { echo "bench $w failed"; tail -20 gpurun_out/fp8_minwork.err; exit 1; }
  tail -1 gpurun_out/fp8_minwork.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('min-work $w', d['value'], d['ms_per_step'], 'fp8', d['config']['fp8_layers'], 'loss', d['config']['final_loss'], flush=True)"
done
