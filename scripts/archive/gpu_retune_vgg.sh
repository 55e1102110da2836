#!/bin/bash
# re-time VGG-16 b2048 bf16 and fp8 GEMM choices after the round-4 DMA changes, A/B the merged DB
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
out=gpurun_out/gemm_tuned_vgg.json
rm -f $out
for dt in bf16 fp8; do
  SN_GEMM_TUNE_DB=0 SN_GEMM_TUNE_PASSES=5 SN_GEMM_TUNE_LOG=1 timeout -k 10 500 python -u bench.py --model vgg16 --dtype $dt --steps 3 --warmup 2 --save-tuned $out > gpurun_out/tune_vgg_$dt.log 2>&1 || { echo "tune $dt failed"; tail -5 gpurun_out/tune_vgg_$dt.log; exit 3; }
  echo "tuned $dt: $(grep -c gemm-tune gpurun_out/tune_vgg_$dt.log) products"
done
python3 - <<'PY'
import json
db = json.load(open("sparknet_amd/ops/gemm_tuned.json"))
new = json.load(open("gpurun_out/gemm_tuned_vgg.json"))
changed = sum(1 for k, v in new.items() if db.get(k) != v)
db.update(new)
json.dump(dict(sorted(db.items())), open("gpurun_out/gemm_tuned_merged_vgg.json", "w"), indent=0)
print(f"retuned {len(new)} products, {changed} changed")
PY
