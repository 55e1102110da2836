#!/bin/bash
# Fill the committed GEMM tuning database with every product of the zoo models' bench
# configurations that it lacks (first-call tuning on an idle GPU, one model at a time),
# then check coverage with autotune off (tests/test_tune_db_gpu.py).  The merged database
# is copied to gpurun_out/gemm_tuned_filled.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
DB=sparknet_amd/ops/gemm_tuned.json
for cfg in "caffenet" "alexnet" "googlenet" "cifar10_quick" "cifar10_full" "vgg16" "vgg16 --dtype fp8"; do
  set -- $cfg
  echo "== $cfg" >> gpurun_out/tune_fill.log
  timeout -k 10 400 python bench.py --model $cfg --steps 2 --warmup 1 > gpurun_out/tf_probe.json 2>> gpurun_out/tune_fill.log || exit 1
  miss=$(python -c "import json;print(json.load(open('gpurun_out/tf_probe.json'))['tune_misses'])")
  echo "misses before: $miss" >> gpurun_out/tune_fill.log
  if [ "$miss" != "0" ]; then
    timeout -k 10 600 python bench.py --model $cfg --steps 2 --warmup 1 --autotune --save-tuned $DB > /dev/null 2>> gpurun_out/tune_fill.log || exit 1
  fi
done
cp $DB gpurun_out/gemm_tuned_filled.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tune_db_gpu.py > gpurun_out/tune_db_tests.log 2>&1
echo "tests rc $?"
cat gpurun_out/tune_fill.log | grep -v amdgpu.ids
tail -12 gpurun_out/tune_db_tests.log
