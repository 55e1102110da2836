#!/bin/bash
# full GPU suite + CaffeNet bench + step trace
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 900 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -12 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc, stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_suite.jsonl 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 5; }
cut -c1-200 gpurun_out/bench_suite.jsonl
exit $rc
