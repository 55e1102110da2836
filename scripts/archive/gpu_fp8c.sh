#!/bin/bash
# fp8 scaling-policy sweep at lr 0.005 (amax history length x margin), 200 VGG-16 steps (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
out=gpurun_out/fp8_policy.txt; : > $out
for noise in ${NOISES:-0.8 0.5}; do
  echo "== noise $noise baseline" >> $out
  timeout -k 10 200 python -u scripts/fp8_trajectory.py --steps 200 --noise $noise --modes bf16,bf16alt >> $out 2>&1 || exit 3
  for pol in "16 1.0" "16 2.0" "0 1.0" "64 1.0"; do
    set -- $pol
    echo "== noise $noise history $1 margin $2" >> $out
    SN_FP8_HISTORY=$1 SN_FP8_MARGIN=$2 timeout -k 10 200 python -u scripts/fp8_trajectory.py --steps 200 --noise $noise --modes bf16,fp8dgw >> $out 2>&1 || exit 4
  done
done
grep -v amdgpu.ids $out
timeout -k 10 300 python -u -m pytest tests/test_gemm_fp8_mc_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/fp8_mc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fp8_mc_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for mode in "--dtype fp8" "--dtype bf16"; do
  timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 $mode >> gpurun_out/vgg_ab2.jsonl 2>> gpurun_out/vgg_ab2.err || { echo "vgg $mode failed"; tail -20 gpurun_out/vgg_ab2.err; exit 5; }
  tail -1 gpurun_out/vgg_ab2.jsonl | cut -c1-200
done
