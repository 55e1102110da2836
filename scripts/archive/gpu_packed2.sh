#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "packed or k96" --timeout 120 --timeout-method thread > gpurun_out/packed2_tests.log 2>&1 || { tail -30 gpurun_out/packed2_tests.log; exit 3; }
tail -1 gpurun_out/packed2_tests.log
for i in 1 2; do timeout -k 10 300 python -u bench.py 2>/dev/null | grep -o '"value": [0-9.]*'; done
rm -rf gpurun_out/prof_pk2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pk2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_pk2.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_pk2.log; exit 5; }
python3 scripts/prof_summary.py gpurun_out/prof_pk2 > gpurun_out/prof_pk2_summary.txt 2>&1
grep -E "^ +[0-9.]+us $|sum of" gpurun_out/prof_pk2_summary.txt
