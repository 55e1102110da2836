#!/bin/bash
# round-5 first call: thin-tile bisection runs, baseline bench, CaffeNet step trace
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for mode in graph eager; do
  timeout -k 10 240 python -u scripts/dbg_thin.py $mode > gpurun_out/dbg_thin_$mode.log 2>&1 || { tail -20 gpurun_out/dbg_thin_$mode.log; exit 3; }
  grep -E "gemm-tune.*M=(32|64) |losses" gpurun_out/dbg_thin_$mode.log | cut -c1-250
done
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r5a.jsonl 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 5; }
tail -1 gpurun_out/bench_r5a.jsonl | cut -c1-200
rm -rf gpurun_out/prof_caffenet
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_caffenet -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/prof_caffenet.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_caffenet.log; exit 6; }
python3 scripts/prof_summary.py gpurun_out/prof_caffenet > gpurun_out/prof_caffenet_summary.txt 2>&1; cat gpurun_out/prof_caffenet_summary.txt
