set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "gemm256" > gpurun_out/ns3_tests.log 2>&1 || { tail -30 gpurun_out/ns3_tests.log; exit 1; }
tail -2 gpurun_out/ns3_tests.log
cp sparknet_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json
APPEND=1 MODELS="caffenet" bash scripts/build_tune_db.sh || exit 1
grep -c . gpurun_out/tune_caffenet.log
for i in 1 2; do
  for db in sparknet_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json; do
    SN_GEMM_TUNE_DB=$db timeout -k 10 300 python bench.py --steps 100 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$db', d['value'], d['ms_per_step'])" || exit 1
  done
done
