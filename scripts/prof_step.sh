# Kernel-trace profile of a short bench.py run: bash scripts/prof_step.sh [bench args...]
# (writes gpurun_out/prof/run_kernel_trace.csv; summarise with scripts/prof_summary.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -rf gpurun_out/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 "$@" > gpurun_out/prof_bench.log 2>&1
