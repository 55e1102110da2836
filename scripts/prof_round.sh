#!/bin/bash
# Kernel-trace profiles of a set of bench configs: bash scripts/prof_round.sh "name|bench args" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; args="${spec#*|}"
  rm -rf gpurun_out/prof_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 $args > gpurun_out/prof_$name.log 2>&1 || { echo "prof $name failed"; tail -5 gpurun_out/prof_$name.log; exit 1; }
  python scripts/prof_summary.py gpurun_out/prof_$name > gpurun_out/prof_${name}_summary.txt 2>&1
  rm -f gpurun_out/prof_$name/run_kernel_trace.csv.gz
  echo "== $name"; tail -1 gpurun_out/prof_${name}_summary.txt
done
