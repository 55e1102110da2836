# fp8-only pooling input gradients (engine.fuse_fp8_quant fp8_dx_only): GPU tests, then VGG-16
# b2048 --dtype fp8 bench.py with the switch on / off, alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_net_gpu.py -k "fp8" \
  tests/test_fp8_fidelity_gpu.py tests/test_fp8_update_gate_gpu.py > gpurun_out/dxonly_tests.log 2>&1 \
  || { tail -40 gpurun_out/dxonly_tests.log; exit 1; }
tail -3 gpurun_out/dxonly_tests.log
: > gpurun_out/dxonly_ab.jsonl
for rep in 1 2; do
  for feat in "" "fp8_dx_only=0"; do
    echo "== rep $rep SN_FEATURES=$feat"
    echo "# rep $rep SN_FEATURES=$feat" >> gpurun_out/dxonly_ab.jsonl
    SN_FEATURES=$feat timeout -k 10 400 python bench.py --model vgg16 --dtype fp8 --steps 20 --warmup 5 \
      >> gpurun_out/dxonly_ab.jsonl 2>> gpurun_out/dxonly_ab.err || { tail -20 gpurun_out/dxonly_ab.err; exit 1; }
    tail -1 gpurun_out/dxonly_ab.jsonl | cut -c1-150
  done
done
