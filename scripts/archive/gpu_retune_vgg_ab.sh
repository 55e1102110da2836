#!/bin/bash
# A/B of a re-timed VGG-16 DB (argument: its path) against the packaged one
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
cand=$1
: > gpurun_out/retune_vgg_ab.txt
for dt in fp8 bf16; do
  for db in new old new old; do
    f=sparknet_amd/ops/gemm_tuned.json; [ $db = new ] && f=$cand
    v=$(SN_GEMM_TUNE_DB=$f timeout -k 10 300 python -u bench.py --model vgg16 --dtype $dt --steps 8 --warmup 3 2>>gpurun_out/retune_vgg.err | grep -o '"value": [0-9.]*') || { tail -5 gpurun_out/retune_vgg.err; exit 4; }
    echo "vgg16 $dt $db $v" | tee -a gpurun_out/retune_vgg_ab.txt
  done
done
