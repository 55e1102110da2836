#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/h2d_probe.py > gpurun_out/h2d.txt 2>&1 || { cat gpurun_out/h2d.txt; exit 3; }
HSA_ENABLE_SDMA=0 timeout -k 10 120 python3 scripts/h2d_probe.py >> gpurun_out/h2d.txt 2>&1 || { cat gpurun_out/h2d.txt; exit 3; }
cat gpurun_out/h2d.txt
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u bench.py > gpurun_out/h2d_bench.jsonl 2> gpurun_out/h2d_bench.err || { tail -5 gpurun_out/h2d_bench.err; exit 4; }
echo "bench SDMA=0: $(cut -c100-200 gpurun_out/h2d_bench.jsonl)"
timeout -k 10 300 python -u bench.py --batch 128 >> gpurun_out/h2d_bench.jsonl 2>> gpurun_out/h2d_bench.err || { tail -5 gpurun_out/h2d_bench.err; exit 4; }
echo "bench b128: $(tail -1 gpurun_out/h2d_bench.jsonl | cut -c100-200)"
