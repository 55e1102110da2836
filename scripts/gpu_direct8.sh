#!/bin/bash
# e4m3 direct conv3x3 (VGG conv1_2): numerics, then VGG-16 b2048 A/B (direct fp8 on / off / bf16), then the lr sweep (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_fp8_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/direct8_tests.log 2>&1
rc=$?; tail -15 gpurun_out/direct8_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/vgg_ab.jsonl
for mode in "--dtype fp8" "--dtype fp8 DIRECT0" "--dtype bf16"; do
  if [ "${mode#*DIRECT0}" != "$mode" ]; then env_d=0; args="--dtype fp8"; else env_d=1; args="$mode"; fi
  SN_CONV_DIRECT_FP8=$env_d timeout -k 10 300 python -u bench.py --model vgg16 --steps ${VGG_STEPS:-8} --warmup 3 $args >> gpurun_out/vgg_ab.jsonl 2>> gpurun_out/vgg_ab.err || { echo "vgg $mode failed"; tail -20 gpurun_out/vgg_ab.err; exit 4; }
  echo "$mode direct=$env_d"; tail -1 gpurun_out/vgg_ab.jsonl | cut -c1-200
done
[ -n "$SKIP_LR" ] || bash scripts/gpu_fp8d.sh
