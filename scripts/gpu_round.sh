#!/bin/bash
# one gpurun call: fp8 lr sweep, CaffeNet bench, full GPU test suite
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
bash scripts/gpu_fp8d.sh || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 5; }
cat gpurun_out/bench.json
bash scripts/gpu_suite.sh
