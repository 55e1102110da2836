# tap-packed conv with magic-number index division (ab/fdiv) vs the integer divisions (ab/base):
# packed-conv tests on the new build, then CaffeNet / GoogLeNet / VGG-16 bf16 benches, alternating
set -o pipefail
mkdir -p gpurun_out
SN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab/fdiv/libsn_kernels.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_kernels_gpu.py tests/test_net_gpu.py -k "packed or fp8_fused" > gpurun_out/fdiv_tests.log 2>&1 \
  || { tail -30 gpurun_out/fdiv_tests.log; exit 1; }
tail -2 gpurun_out/fdiv_tests.log
: > gpurun_out/fdiv_ab.txt
for rep in 1 2 3; do
  for v in fdiv base; do
    export SN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab/$v/libsn_kernels.so
    for m in caffenet googlenet vgg16; do
      st=50; [ $m = vgg16 ] && st=15
      timeout -k 10 400 python bench.py --model $m --steps $st --warmup 5 2>/dev/null > gpurun_out/fdiv_one.json || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/fdiv_one.json').read().strip().splitlines()[-1]); print('$v', '$m', d['value'], d['ms_per_step'])" | tee -a gpurun_out/fdiv_ab.txt
    done
  done
done
