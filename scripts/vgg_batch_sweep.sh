#!/bin/bash
# VGG-16 throughput and peak device memory vs per-GPU batch (BASELINE config 5: batch sized
# for 288 GB of HBM), bf16 and fp8 forward products.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 64 128 256 512; do
  for dt in bf16 fp8; do
    timeout -k 10 300 python bench.py --model vgg16 --batch $b --dtype $dt --steps 10 --warmup 4 > gpurun_out/vgg_${b}_${dt}.json 2>gpurun_out/vgg_${b}_${dt}.err || { echo "batch $b $dt failed"; tail -3 gpurun_out/vgg_${b}_${dt}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/vgg_${b}_${dt}.json')); print('batch', $b, '$dt', d['value'], 'img/s', d['ms_per_step'], 'ms', d['max_mem_gb'], 'GB')"
  done
done
