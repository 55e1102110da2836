#!/bin/bash
# native capi tests, bench-config fidelity gate, CaffeNet step trace (per launch)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_core_capi.py -m gpu > gpurun_out/capi_gpu.log 2>&1 || { tail -30 gpurun_out/capi_gpu.log; exit 3; }
tail -3 gpurun_out/capi_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cn5 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_cn5.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_cn5.log; exit 5; }
f=$(ls gpurun_out/prof_cn5/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_cn5/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_cn5_summary.txt && head -40 gpurun_out/prof_cn5_summary.txt
rm -rf gpurun_out/prof_cn5
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_bench_fidelity_gpu.py -m gpu > gpurun_out/fid_gpu.log 2>&1; rc=$?
grep -E "per-parameter|PASS|FAIL|Error|passed|failed" gpurun_out/fid_gpu.log | cut -c1-1500 | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

