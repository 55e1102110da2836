#!/bin/bash
# re-time CaffeNet / GoogLeNet GEMM choices after the round-4 DMA changes, then A/B the merged DB
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
MODELS="caffenet googlenet" bash scripts/build_tune_db.sh || exit 3
python3 - <<'PY'
import json
db = json.load(open("sparknet_amd/ops/gemm_tuned.json"))
new = json.load(open("gpurun_out/gemm_tuned.json"))
changed = sum(1 for k, v in new.items() if db.get(k) != v)
db.update(new)
json.dump(dict(sorted(db.items())), open("gpurun_out/gemm_tuned_merged.json", "w"), indent=0)
print(f"retuned {len(new)} products, {changed} changed")
PY
: > gpurun_out/retune_ab.jsonl
for m in caffenet googlenet; do
  for db in new old new old; do
    f=sparknet_amd/ops/gemm_tuned.json; [ $db = new ] && f=gpurun_out/gemm_tuned_merged.json
    SN_GEMM_TUNE_DB=$f timeout -k 10 300 python -u bench.py --model $m >> gpurun_out/retune_ab.jsonl 2> gpurun_out/retune_ab.err || { tail -5 gpurun_out/retune_ab.err; exit 4; }
    echo "$m $db $(tail -1 gpurun_out/retune_ab.jsonl | grep -o '"value": [0-9.]*')"
  done
done
