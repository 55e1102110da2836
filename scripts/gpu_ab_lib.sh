# same-box A/B of two kernel builds (ab/base vs ab/pipe2): conv probe + benches, alternating
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_lib.txt
for rep in 1 2; do
  for v in base pipe2; do
    export SN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab/$v/libsn_kernels.so
    echo "== $v rep $rep" >> gpurun_out/ab_lib.txt
    timeout -k 10 200 python -u scripts/conv_probe.py --case cn_conv2g,cn_conv3,cn_conv5g,gn_3b_3x3 --tiles=-1,0 --no-dense >> gpurun_out/ab_lib.txt 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/ab_lib.txt; exit 1; }
    timeout -k 10 200 python bench.py >> gpurun_out/ab_lib.txt 2>/dev/null || { echo "bench $v failed"; exit 1; }
    timeout -k 10 200 python bench.py --model googlenet >> gpurun_out/ab_lib.txt 2>/dev/null || { echo "bench gn $v failed"; exit 1; }
  done
done
grep -v amdgpu gpurun_out/ab_lib.txt | cut -c1-160
