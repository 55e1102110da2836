# round-end validation: GPU suite + smoke + bench (gpu_suite_smoke.sh), then PMC passes over a CaffeNet bench step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_suite_smoke.sh || exit 1
PROG=bench.py PROG_ARGS="--steps 2 --warmup 1" bash scripts/pmc_passes.sh > gpurun_out/final_pmc.log 2>&1 || { tail -5 gpurun_out/final_pmc.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/final_pmc_summary.txt 2>&1; head -50 gpurun_out/final_pmc_summary.txt
