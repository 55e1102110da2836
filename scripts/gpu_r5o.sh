#!/bin/bash
# full GPU suite, then CaffeNet bench sweep of the fused LRN+pool backward tile (SN_PLRN_CG / SN_PLRN_LDS)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 800 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc, stopping"; exit $rc; fi
: > gpurun_out/plrn_ab.jsonl
for cfg in "base" "SN_PLRN_LDS=65536" "SN_PLRN_CG=12" "SN_PLRN_CG=6" "SN_PLRN_LDS=16384" "base"; do
  if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
  env $e timeout -k 10 300 python -u bench.py >> gpurun_out/plrn_ab.jsonl 2> gpurun_out/plrn_ab.err || { tail -20 gpurun_out/plrn_ab.err; exit 5; }
  echo "$cfg: $(tail -1 gpurun_out/plrn_ab.jsonl | cut -c70-130)"
done
exit $rc
