#!/bin/bash
# same-box A/B of the lean MC im2col (weight-gradient) address path (SN_GEMM_LEGACY_ADDR=2 turns it
# off), CaffeNet bench both ways, VGG-16 b2048 fp8 (direct conv1_2 on / off) vs bf16, PMC of conv3
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "conv or fast_dma or small_cg" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log
[ $rc -eq 0 ] || exit $rc
for L in 0 2; do
  SN_GEMM_LEGACY_ADDR=$L timeout -k 10 400 python -u scripts/pk_probe.py --model caffenet --tiles '' > gpurun_out/ab_census_$L.txt 2>&1 || { tail -20 gpurun_out/ab_census_$L.txt; exit 3; }
  tail -1 gpurun_out/ab_census_$L.txt
done
for L in 0 2 0; do
  SN_GEMM_LEGACY_ADDR=$L timeout -k 10 300 python -u bench.py >> gpurun_out/ab_bench.jsonl 2>> gpurun_out/ab_bench.err || { tail -20 gpurun_out/ab_bench.err; exit 5; }
  echo "legacy=$L $(tail -1 gpurun_out/ab_bench.jsonl | cut -c1-130)"
done
: > gpurun_out/vgg_ab.jsonl
for mode in "--dtype fp8" "--dtype fp8 DIRECT0" "--dtype bf16"; do
  if [ "${mode#*DIRECT0}" != "$mode" ]; then env_d=0; args="--dtype fp8"; else env_d=1; args="$mode"; fi
  SN_CONV_DIRECT_FP8=$env_d timeout -k 10 300 python -u bench.py --model vgg16 --steps ${VGG_STEPS:-8} --warmup 3 $args >> gpurun_out/vgg_ab.jsonl 2>> gpurun_out/vgg_ab.err || { echo "vgg $mode failed"; tail -20 gpurun_out/vgg_ab.err; exit 4; }
  echo "$mode direct=$env_d"; tail -1 gpurun_out/vgg_ab.jsonl | cut -c1-160
done
TILES=0 WGRAD_TILES=0 bash scripts/pmc_tiles.sh > gpurun_out/ab_pmc.log 2>&1 || { tail -20 gpurun_out/ab_pmc.log; exit 6; }
tail -12 gpurun_out/ab_pmc.log
