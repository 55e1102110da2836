#!/bin/bash
# Re-tune the CaffeNet / GoogLeNet GEMM entries from scratch on this box (9 passes), then A/B
# the packaged database against the fresh one (driver-shaped benches, interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
MODELS="caffenet googlenet" bash scripts/build_tune_db.sh || exit 1
for r in 1 2 3; do
  for db in packaged fresh; do
    if [ $db = fresh ]; then export SN_GEMM_TUNE_DB=$GRAFT_REPO_ROOT/gpurun_out/gemm_tuned.json; else unset SN_GEMM_TUNE_DB; fi
    for m in caffenet googlenet; do
      timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m db=$db', d['value'], d['ms_per_step'], flush=True)" || exit 1
    done
  done
done
