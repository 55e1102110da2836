#!/bin/bash
# merged Inception siblings: numerics, then GoogLeNet A/B (SN_FUSE_SIBLINGS 1 / 0, interleaved)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_siblings_gpu.py -x -q -s -rf --timeout 300 --timeout-method thread > gpurun_out/sib_tests.log 2>&1
rc=$?; tail -15 gpurun_out/sib_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/sib_ab.jsonl
for i in 1 2; do
  for f in 1 0; do
    SN_FUSE_SIBLINGS=$f timeout -k 10 300 python -u bench.py --model googlenet --steps 20 --warmup 5 >> gpurun_out/sib_ab.jsonl 2> gpurun_out/sib_ab.err || { tail -20 gpurun_out/sib_ab.err; exit 5; }
    echo "siblings=$f $(tail -1 gpurun_out/sib_ab.jsonl | cut -c1-120)"
  done
done
