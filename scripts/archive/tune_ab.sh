#!/bin/bash
# Retune one model's GEMMs from scratch (new kernel candidates), then bench the packaged
# tuning database against the fresh one on the same box, alternating.
#   MODEL=caffenet bash scripts/tune_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
M=${MODEL:-caffenet}
out=gpurun_out/tuned_$M.json
rm -f $out
SN_GEMM_TUNE_DB=0 SN_GEMM_TUNE_PASSES=9 SN_GEMM_TUNE_LOG=1 timeout -k 10 600 python bench.py --model $M --steps 4 --warmup 3 --save-tuned $out > gpurun_out/tune_$M.log 2>&1 || { echo "tune failed"; tail -5 gpurun_out/tune_$M.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --model $M --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('packaged', d['value'], d['ms_per_step'])"
  SN_GEMM_TUNE_DB=$out timeout -k 10 300 python bench.py --model $M --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fresh   ', d['value'], d['ms_per_step'])"
done
