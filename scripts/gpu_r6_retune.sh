#!/bin/bash
# r6: re-time the conv weight-gradient products after the MC im2col stager change (their
# database entries were measured on the old stager), fill any other misses, check coverage,
# then bench CaffeNet / GoogLeNet on the new database.  The database lands in
# gpurun_out/gemm_tuned_r6.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
DB=sparknet_amd/ops/gemm_tuned.json
python scripts/tune_db_strip.py $DB wgrad > gpurun_out/r6r_tune.log || exit 1
for cfg in "caffenet" "alexnet" "googlenet" "cifar10_quick" "cifar10_full" "vgg16" "vgg16 --dtype fp8"; do
  echo "== $cfg" >> gpurun_out/r6r_tune.log
  timeout -k 10 600 python bench.py --model $cfg --steps 2 --warmup 1 --autotune --save-tuned $DB > gpurun_out/r6r_fill.json 2>> gpurun_out/r6r_tune.log || { echo "tune failed: $cfg"; tail -20 gpurun_out/r6r_tune.log; exit 1; }
  cp $DB gpurun_out/gemm_tuned_r6.json
done
grep -v amdgpu.ids gpurun_out/r6r_tune.log | tail -20
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_tune_db_gpu.py > gpurun_out/r6r_tests.log 2>&1; echo "tune-db tests rc $?"; tail -3 gpurun_out/r6r_tests.log
for i in 1 2; do timeout -k 10 240 python bench.py > gpurun_out/r6r_bench$i.json 2>/dev/null || exit 1; cut -c1-150 gpurun_out/r6r_bench$i.json; done
timeout -k 10 240 python bench.py --model googlenet > gpurun_out/r6r_gn.json 2>/dev/null || exit 1; cut -c1-150 gpurun_out/r6r_gn.json
