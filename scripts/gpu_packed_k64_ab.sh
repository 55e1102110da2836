# VGG-16 conv1_1 on the tap-packed <3, 64> kernel: kernel tests, then VGG-16 b2048 bf16 / fp8 benches with
# SN_FEATURES=conv_packed_k64 on / off, alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_net_gpu.py tests/test_fp8_update_gate_gpu.py -k "packed or fp8" \
  > gpurun_out/k64_tests.log 2>&1 || { tail -30 gpurun_out/k64_tests.log; exit 1; }
tail -2 gpurun_out/k64_tests.log
: > gpurun_out/k64_ab.jsonl
for rep in 1 2; do
  for dt in bf16 fp8; do
    for feat in "" "conv_packed_k64=0"; do
      echo "== rep $rep $dt SN_FEATURES=$feat"
      echo "# rep $rep $dt SN_FEATURES=$feat" >> gpurun_out/k64_ab.jsonl
      SN_FEATURES=$feat timeout -k 10 400 python bench.py --model vgg16 --dtype $dt --steps 20 --warmup 5 \
        >> gpurun_out/k64_ab.jsonl 2>> gpurun_out/k64_ab.err || { tail -20 gpurun_out/k64_ab.err; exit 1; }
      tail -1 gpurun_out/k64_ab.jsonl | cut -c1-130
    done
  done
done
