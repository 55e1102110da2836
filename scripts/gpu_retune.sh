#!/bin/bash
# r6: re-time the conv weight-gradient products after the MC im2col stager change (their
# database entries were measured on the old stager) and fill any other misses, model by
# model (MODELS="caffenet|googlenet|..."; STRIP=1 drops the wgrad entries first); the merged
# database lands in gpurun_out/gemm_tuned_r6.json.  CHECK=1 then runs the coverage /
# reproducibility tests and benches CaffeNet and GoogLeNet on it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
DB=sparknet_amd/ops/gemm_tuned.json
[ -f gpurun_out/gemm_tuned_r6.json ] && cp gpurun_out/gemm_tuned_r6.json $DB
[ "$STRIP" = "1" ] && { python scripts/tune_db_strip.py $DB wgrad >> gpurun_out/r6r_tune.log || exit 1; }
# heartbeat: the first VGG-16 b2048 tuning steps print nothing for minutes
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
IFS='|' read -ra CFGS <<< "$MODELS"
for cfg in "${CFGS[@]}"; do
  [ -z "$cfg" ] && continue
  echo "== $cfg" >> gpurun_out/r6r_tune.log
  timeout -k 10 500 python bench.py --model $cfg --steps 2 --warmup 1 --autotune --save-tuned $DB > gpurun_out/r6r_fill.json 2>> gpurun_out/r6r_tune.log || { echo "tune failed: $cfg"; tail -20 gpurun_out/r6r_tune.log; exit 1; }
  cp $DB gpurun_out/gemm_tuned_r6.json
  echo "$cfg done"
done
grep -v amdgpu.ids gpurun_out/r6r_tune.log | tail -12
if [ "$CHECK" = "1" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_tune_db_gpu.py > gpurun_out/r6r_tests.log 2>&1; echo "tune-db tests rc $?"; tail -3 gpurun_out/r6r_tests.log
  for i in 1 2; do timeout -k 10 240 python bench.py > gpurun_out/r6r_bench$i.json 2>/dev/null || exit 1; cut -c1-150 gpurun_out/r6r_bench$i.json; done
  timeout -k 10 240 python bench.py --model googlenet > gpurun_out/r6r_gn.json 2>/dev/null || exit 1; cut -c1-150 gpurun_out/r6r_gn.json
fi
