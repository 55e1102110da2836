# round 6: the full GPU suite (as the driver runs it), smoke(), then one bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread > gpurun_out/r6s_gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r6s_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r6s_smoke.log; exit 1; }
tail -3 gpurun_out/r6s_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6s_bench.json 2> gpurun_out/r6s_bench.err || { echo bench failed; tail -20 gpurun_out/r6s_bench.err; exit 1; }
cut -c1-200 gpurun_out/r6s_bench.json
