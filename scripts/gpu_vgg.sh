#!/bin/bash
# VGG-16 b2048 fp8 (direct conv1_2 on / off) vs bf16, then the conv3 PMC passes (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/vgg_ab.jsonl; : > gpurun_out/vgg_ab.err
for mode in "--dtype fp8" "--dtype fp8 DIRECT0" "--dtype bf16"; do
  if [ "${mode#*DIRECT0}" != "$mode" ]; then env_d=0; args="--dtype fp8"; else env_d=1; args="$mode"; fi
  SN_CONV_DIRECT_FP8=$env_d timeout -k 10 300 python -u bench.py --model vgg16 --steps ${VGG_STEPS:-8} --warmup 3 $args >> gpurun_out/vgg_ab.jsonl 2>> gpurun_out/vgg_ab.err || { echo "vgg $mode failed"; tail -5 gpurun_out/vgg_ab.err; exit 4; }
  echo "$mode direct=$env_d"; tail -1 gpurun_out/vgg_ab.jsonl | cut -c1-160
done
TILES=0 WGRAD_TILES=0 bash scripts/pmc_tiles.sh > gpurun_out/ab_pmc.log 2>&1 || { tail -20 gpurun_out/ab_pmc.log; exit 6; }
tail -12 gpurun_out/ab_pmc.log
