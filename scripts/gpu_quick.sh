#!/bin/bash
# Targeted GPU tests (args: pytest node ids / -k expressions), then the 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/quick_tests.log 2>&1 || { echo "quick tests failed"; tail -60 gpurun_out/quick_tests.log; exit 1; }
tail -3 gpurun_out/quick_tests.log
