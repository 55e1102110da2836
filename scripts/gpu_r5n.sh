#!/bin/bash
# split-K combine (write-through slabs): tests, per-product CaffeNet census off / heuristic /
# always, CaffeNet + GoogLeNet bench A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_splitk_fixup_gpu.py -m gpu > gpurun_out/fix_tests.log 2>&1 || { tail -40 gpurun_out/fix_tests.log; exit 3; }
tail -1 gpurun_out/fix_tests.log
for fx in 0 1 2; do
  SN_GEMM_FIXUP=$fx timeout -k 10 300 python -u scripts/pk_probe.py --model caffenet --tiles "" > gpurun_out/census_fix$fx.txt 2>&1 || { tail -20 gpurun_out/census_fix$fx.txt; exit 4; }
done
paste <(grep -E "fwd|bwd|total" gpurun_out/census_fix0.txt | cut -c1-75) <(grep -E "fwd|bwd|total" gpurun_out/census_fix1.txt | cut -c60-75) <(grep -E "fwd|bwd|total" gpurun_out/census_fix2.txt | cut -c60-75)
: > gpurun_out/fix_ab.jsonl
for i in 1 2; do
  for fx in 0 1; do
    SN_GEMM_FIXUP=$fx timeout -k 10 300 python -u bench.py >> gpurun_out/fix_ab.jsonl 2> gpurun_out/fix_ab.err || { tail -20 gpurun_out/fix_ab.err; exit 5; }
    echo "caffenet fixup=$fx: $(tail -1 gpurun_out/fix_ab.jsonl | cut -c70-130)"
  done
done
for i in 1 2; do
  for fx in 0 1; do
    SN_GEMM_FIXUP=$fx timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/fix_ab.jsonl 2> gpurun_out/fix_ab.err || { tail -20 gpurun_out/fix_ab.err; exit 5; }
    echo "googlenet fixup=$fx: $(tail -1 gpurun_out/fix_ab.jsonl | cut -c1-60)"
  done
done
