#!/bin/bash
# LDS-band 3x3/s1 max pool: kernel tests, isolated probe (band vs gathers), GoogLeNet bench A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "pool" > gpurun_out/aj_tests.log 2>&1 || { tail -40 gpurun_out/aj_tests.log; exit 3; }
tail -1 gpurun_out/aj_tests.log
for v in 1 0; do
  SN_POOL_BAND=$v timeout -k 10 300 python -u scripts/pool_probe.py --batch 128 --only "gn" > gpurun_out/aj_probe$v.txt 2>&1 || { tail -20 gpurun_out/aj_probe$v.txt; exit 4; }
  echo "band=$v"; grep -v amdgpu.ids gpurun_out/aj_probe$v.txt
done
: > gpurun_out/aj_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    SN_POOL_BAND=$v timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/aj_ab.jsonl 2> gpurun_out/aj_ab.err || { tail -20 gpurun_out/aj_ab.err; exit 5; }
    echo "googlenet band=$v: $(tail -1 gpurun_out/aj_ab.jsonl | cut -c45-75)"
  done
done
