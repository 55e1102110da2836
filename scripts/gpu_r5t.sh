#!/bin/bash
# VGG-16 b2048 fp8 vs bf16, interleaved (BASELINE configs[4] shape), plus AlexNet / cifar smoke numbers
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/vgg5.jsonl
for dt in fp8 bf16 fp8 bf16; do
  timeout -k 10 500 python -u bench.py --model vgg16 --dtype $dt --steps 6 --warmup 3 >> gpurun_out/vgg5.jsonl 2> gpurun_out/vgg5.err || { tail -20 gpurun_out/vgg5.err; exit 5; }
  echo "vgg16 $dt: $(tail -1 gpurun_out/vgg5.jsonl | cut -c1-75)"
done
