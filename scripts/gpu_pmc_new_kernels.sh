# PMC passes (scripts/pmc_passes.sh) over one AlexNet bench step (pool_lrn_bwd_rev) and one small VGG-16 step
# (conv_packed <3, 64>), summaries by scripts/pmc_summary.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PROG=bench.py PROG_ARGS="--model alexnet --steps 2 --warmup 1" bash scripts/pmc_passes.sh > gpurun_out/pmc_alex.log 2>&1 || { tail -5 gpurun_out/pmc_alex.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_alex_summary.txt 2>&1
grep -E "pool_lrn_bwd_rev|lrn_across_fwd|maxpool_fwd" gpurun_out/pmc_alex_summary.txt | cut -c1-400
rm -rf gpurun_out/pmc
PROG=bench.py PROG_ARGS="--model vgg16 --batch 256 --steps 2 --warmup 1" bash scripts/pmc_passes.sh > gpurun_out/pmc_vgg.log 2>&1 || { tail -5 gpurun_out/pmc_vgg.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_vgg_summary.txt 2>&1
grep -E "conv_packed|conv3x3" gpurun_out/pmc_vgg_summary.txt | cut -c1-400
rm -rf gpurun_out/pmc
