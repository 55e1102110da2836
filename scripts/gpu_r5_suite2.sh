#!/bin/bash
# full GPU suite only (final tree)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 900 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; tail -6 gpurun_out/gpu_tests_final.log; exit $rc
