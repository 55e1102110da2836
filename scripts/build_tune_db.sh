#!/bin/bash
# Offline GEMM tuning database for the benchmark models (run on an MI355X box):
#   bash scripts/build_tune_db.sh   -> gpurun_out/gemm_tuned.json
#   (MODELS="vgg16 cifar10_quick" APPEND=1 bash scripts/build_tune_db.sh adds to it)
# then copy it to sparknet_amd/ops/gemm_tuned.json.  Every product is timed from scratch
# (the packaged database is ignored) with 9 interleaved passes per candidate.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/gemm_tuned.json
[ -n "$APPEND" ] || rm -f $out
export SN_GEMM_TUNE_DB=0 SN_GEMM_TUNE_PASSES=9 SN_GEMM_TUNE_LOG=1  # the log lines also keep the run visibly alive
MODELS=${MODELS:-"caffenet googlenet vgg16 cifar10_quick cifar10_full"}
for spec in $MODELS; do
  timeout -k 10 900 python bench.py --model $spec --steps 4 --warmup 3 --save-tuned $out > gpurun_out/tune_$(echo $spec | tr ' ' '_').log 2>&1 || { echo "tune $spec failed"; tail -5 gpurun_out/tune_*.log; exit 1; }
  echo "tuned $spec: $(tail -1 gpurun_out/tune_$(echo $spec | tr ' ' '_').log)"
done
