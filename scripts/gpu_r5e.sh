#!/bin/bash
# GoogLeNet: bench, kernel trace, per-product GEMM census (tuned configs only)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model googlenet --steps 20 --warmup 5 > gpurun_out/gn_bench.jsonl 2> gpurun_out/gn_bench.err || { tail -20 gpurun_out/gn_bench.err; exit 5; }
cut -c1-200 gpurun_out/gn_bench.jsonl
rm -rf gpurun_out/prof_gn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gn -o run --output-format csv -- python3 bench.py --model googlenet --steps 6 --warmup 3 > gpurun_out/prof_gn.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_gn.log; exit 6; }
python3 scripts/prof_summary.py gpurun_out/prof_gn > gpurun_out/prof_gn_summary.txt 2>&1; cat gpurun_out/prof_gn_summary.txt
timeout -k 10 400 python -u scripts/pk_probe.py --model googlenet --tiles "" > gpurun_out/gn_census.txt 2>&1 || { tail -20 gpurun_out/gn_census.txt; exit 3; }
tail -3 gpurun_out/gn_census.txt
