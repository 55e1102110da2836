#!/bin/bash
# A/B of bench.py under env settings, interleaved: bash scripts/ab_bench_env.sh "VAR=a" "VAR=b" [rounds] [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
A=$1; B=$2; R=${3:-2}; shift 3
mkdir -p gpurun_out
for r in $(seq $R); do
  for e in "$A" "$B"; do
    out=$(env $e timeout -k 10 300 python bench.py --steps 50 --warmup 10 "$@" 2>/dev/null) || { echo "bench failed ($e)"; exit 1; }
    echo "$e $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])')"
  done
done
