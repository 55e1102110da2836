# tap-packed conv: LDS-staged coalesced output stores vs fragment-layout stores (ab/base vs ab/stage
# builds), packed-conv tests on the staged build, then VGG-16 bf16 / GoogLeNet benches alternating
set -o pipefail
mkdir -p gpurun_out
SN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab/stage/libsn_kernels.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_kernels_gpu.py tests/test_net_gpu.py -k "packed or fp8_fused" > gpurun_out/stage_tests.log 2>&1 \
  || { tail -30 gpurun_out/stage_tests.log; exit 1; }
tail -2 gpurun_out/stage_tests.log
: > gpurun_out/stage_ab.txt
for rep in 1 2; do
  for v in stage base; do
    export SN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab/$v/libsn_kernels.so
    for m in vgg16 googlenet; do
      timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 2>/dev/null > gpurun_out/stage_one.json || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/stage_one.json').read().strip().splitlines()[-1]); print('$v', '$m', d['value'], d['ms_per_step'])" | tee -a gpurun_out/stage_ab.txt
    done
  done
done
