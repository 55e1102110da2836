#!/bin/bash
# GoogLeNet GEMM census aggregated per Inception branch type (isolated launch times)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python scripts/gemm_census.py --model googlenet --reps 10 > gpurun_out/census_googlenet.txt 2>&1 || exit 1
tail -1 gpurun_out/census_googlenet.txt
grep -E "inception" gpurun_out/census_googlenet.txt | awk '{split($1,a,":"); l=a[1]; sub(/.*\//,"",l); t[l]+=$(NF-1)} END {for (k in t) printf "%-14s %8.1f\n", k, t[k]}' | sort -k2 -nr
