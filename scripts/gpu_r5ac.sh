#!/bin/bash
# fp8 weight-gradient bias: exact bf16 column sum (default) vs the e4m3 ones column on the
# quantised dy — fidelity gate and VGG-16 b2048 fp8 throughput, both modes
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for b in 0 1; do
  SN_FP8_WGRAD_BIAS=$b timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread tests/test_fp8_fidelity_gpu.py -m gpu > gpurun_out/fp8bias_fid_$b.log 2>&1; rc=$?
  echo "bias mode $b fidelity rc=$rc: $(grep -E "passed|failed" gpurun_out/fp8bias_fid_$b.log | tail -1)"; grep -iE "deviation|floor|max|smoothed" gpurun_out/fp8bias_fid_$b.log | tail -4 | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
: > gpurun_out/fp8bias_bench.jsonl
for b in 1 0 1 0; do
  SN_FP8_WGRAD_BIAS=$b timeout -k 10 500 python -u bench.py --model vgg16 --dtype fp8 --steps 6 --warmup 3 >> gpurun_out/fp8bias_bench.jsonl 2> gpurun_out/fp8bias_bench.err || { tail -20 gpurun_out/fp8bias_bench.err; exit 5; }
  echo "vgg16 fp8 bias=$b: $(tail -1 gpurun_out/fp8bias_bench.jsonl | cut -c1-75)"
done
