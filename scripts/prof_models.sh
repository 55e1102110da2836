# Kernel-trace profiles of the other zoo models: bash scripts/prof_models.sh model [model...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for m in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python3 bench.py --model $m --steps 6 --warmup 3 > gpurun_out/prof_$m.log 2>&1 || exit 1
  python scripts/prof_summary.py gpurun_out/prof_$m all > gpurun_out/prof_${m}_summary.txt 2>&1
done
