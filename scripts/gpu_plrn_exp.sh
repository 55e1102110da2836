# same-box A/B of pool+LRN backward builds under ab/<variant>/ (plrn_probe + CaffeNet bench), alternating
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/plrn_exp.txt
for rep in 1 2; do
  for v in base fold foldpk; do
    echo "== $v rep $rep" >> gpurun_out/plrn_exp.txt
    export SN_KERNEL_LIB=$GRAFT_REPO_ROOT/ab/$v/libsn_kernels.so
    timeout -k 10 120 python -u scripts/plrn_probe.py >> gpurun_out/plrn_exp.txt 2>&1 || { tail -5 gpurun_out/plrn_exp.txt; exit 1; }
    timeout -k 10 200 python bench.py 2>/dev/null | cut -c1-140 >> gpurun_out/plrn_exp.txt || { echo "bench $v failed"; exit 1; }
  done
done
grep -v amdgpu gpurun_out/plrn_exp.txt
