# LRN -> max-pool backward fusion (engine.fuse_lrn_pool_backward): GPU tests, then AlexNet and
# GoogLeNet bench.py with the fusion on / off, alternating on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_pool_lrn_gpu.py \
  > gpurun_out/lrnrev_tests.log 2>&1 || { tail -30 gpurun_out/lrnrev_tests.log; exit 1; }
tail -3 gpurun_out/lrnrev_tests.log
timeout -k 10 120 python scripts/plrn_rev_probe.py > gpurun_out/lrnrev_probe.txt 2>&1 || { tail -20 gpurun_out/lrnrev_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/lrnrev_probe.txt
: > gpurun_out/lrnrev_ab.jsonl
for rep in 1 2; do
  for model in alexnet googlenet; do
    for feat in "" "fuse_lrn_pool_bwd=0"; do
      echo "== $model rep $rep SN_FEATURES=$feat"
      echo "# $model rep $rep SN_FEATURES=$feat" >> gpurun_out/lrnrev_ab.jsonl
      SN_FEATURES=$feat timeout -k 10 240 python bench.py --model $model --steps 40 --warmup 10 \
        >> gpurun_out/lrnrev_ab.jsonl 2>> gpurun_out/lrnrev_ab.err || exit 1
      tail -1 gpurun_out/lrnrev_ab.jsonl | cut -c1-160
    done
  done
done
