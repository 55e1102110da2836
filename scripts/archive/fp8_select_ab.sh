#!/bin/bash
# VGG-16 (batch 512) fp8 layer selection A/B: bf16 vs fp8 at several min-MACs-per-input thresholds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/fp8_select.jsonl
for spec in "--dtype bf16" "--dtype fp8 --fp8-min-work 0" "--dtype fp8 --fp8-min-work 1000" "--dtype fp8 --fp8-min-work 2000" \
            "--dtype fp8 --fp8-min-work 4000" "--dtype bf16" "--dtype fp8 --fp8-min-work 2000"; do
  timeout -k 10 300 python bench.py --model vgg16 --steps 10 --warmup 3 $spec >> gpurun_out/fp8_select.jsonl 2> gpurun_out/fp8_select.err || { echo "bench $spec failed"; tail -20 gpurun_out/fp8_select.err; exit 1; }
  tail -1 gpurun_out/fp8_select.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], 'fp8_layers', d['config']['fp8_layers'], 'loss', d['config']['final_loss'], flush=True)"
done
