#!/bin/bash
# VGG-16 b2048 fp8 variants (direct e4m3 conv1_2; 64-row thin tiles), then kernel traces (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/vgg_var.jsonl
for v in "SN_CONV_DIRECT_FP8=1" "SN_GEMM_THIN=1" "SN_CONV_DIRECT_FP8=1 SN_GEMM_THIN=1"; do
  env $v timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 --dtype fp8 >> gpurun_out/vgg_var.jsonl 2> gpurun_out/vgg_var.err
  rc=$?; echo "== $v rc=$rc $(tail -1 gpurun_out/vgg_var.jsonl | cut -c1-150)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -3 gpurun_out/vgg_var.err; exit $rc; fi
done
bash scripts/gpu_prof.sh
