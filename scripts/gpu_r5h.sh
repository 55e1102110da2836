#!/bin/bash
# merged siblings: GoogLeNet kernel traces with and without
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for f in 1 0; do
  rm -rf gpurun_out/prof_sib$f
  SN_FUSE_SIBLINGS=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sib$f -o run --output-format csv -- python3 bench.py --model googlenet --steps 6 --warmup 3 > gpurun_out/prof_sib$f.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_sib$f.log; exit 6; }
  python3 scripts/prof_summary.py gpurun_out/prof_sib$f > gpurun_out/prof_sib${f}_summary.txt 2>&1; echo "== siblings=$f"; head -30 gpurun_out/prof_sib${f}_summary.txt; tail -1 gpurun_out/prof_sib${f}_summary.txt
done
