#!/bin/bash
# Split-K cap A/B (SN_GEMM_MAX_SPLITS): GoogLeNet b128 (4 branch streams) and CaffeNet, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CAPVAR=${CAPVAR:-SN_GEMM_MAX_SPLITS}; CAPS=${CAPS:-"0 1 4 0 1"}
for m in ${MODELS:-googlenet caffenet}; do
  for cap in $CAPS; do
    env $CAPVAR=$cap timeout -k 10 240 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/sk_$m$cap.json 2> gpurun_out/sk_$m$cap.err || { echo "bench $m cap $cap failed"; tail -20 gpurun_out/sk_$m$cap.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sk_$m$cap.json')); print('$m max_splits=$cap', d['value'], d['ms_per_step'], flush=True)"
  done
done
