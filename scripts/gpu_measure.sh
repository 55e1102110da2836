#!/bin/bash
# r6: PMC passes on CaffeNet conv3 forward (tile 0) and weight gradient (tiles 0 / 10) with the
# lean MC stager, the forward im2col-vs-dense probe for conv2 / conv5 groups, then kernel traces
# of one CaffeNet and one GoogLeNet step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
[ -f gpurun_out/gemm_tuned_r6.json ] && cp gpurun_out/gemm_tuned_r6.json sparknet_amd/ops/gemm_tuned.json
TILES=0 WGRAD_TILES=0,10 bash scripts/pmc_tiles.sh > gpurun_out/r6m_pmc.txt 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/r6m_pmc.txt; exit 1; }
tail -40 gpurun_out/r6m_pmc.txt
bash scripts/pmc_blas.sh > gpurun_out/r6m_pmc_blas.txt 2>&1 || { echo "pmc blas failed"; tail -20 gpurun_out/r6m_pmc_blas.txt; exit 1; }
tail -60 gpurun_out/r6m_pmc_blas.txt
timeout -k 10 300 python -u scripts/conv_probe.py --case cn_conv2g,cn_conv5g,cn_conv3 --tiles=-1,0,13,16,17 > gpurun_out/r6m_conv.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r6m_conv.txt
run() {  # name, bench args...
  local n=$1; shift
  rm -rf gpurun_out/prof_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run --output-format csv -- python3 bench.py --steps 4 --warmup 3 "$@" > gpurun_out/prof_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/prof_$n.log; return 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_$n all > gpurun_out/prof_${n}_summary.txt 2>&1
  head -30 gpurun_out/prof_${n}_summary.txt
}
run r6caffenet && run r6googlenet --model googlenet && run r6vggfp8 --model vgg16 --dtype fp8
rm -rf gpurun_out/prof_r6caffenet/*/ gpurun_out/prof_r6googlenet/*/ gpurun_out/prof_r6vggfp8/*/ 2>/dev/null; true
