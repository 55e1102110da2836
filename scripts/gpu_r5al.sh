#!/bin/bash
# LRN s^-beta on raw v_log/v_exp: LRN + fused pool/LRN tests, isolated kernel probe, CaffeNet + GoogLeNet benches, CaffeNet step trace
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_pool_lrn_gpu.py tests/test_gradcheck.py -m gpu -k "lrn or LRN or pool" > gpurun_out/al_tests.log 2>&1 || { tail -40 gpurun_out/al_tests.log; exit 3; }
tail -1 gpurun_out/al_tests.log
timeout -k 10 200 python -u scripts/plrn_probe.py 32768 > gpurun_out/al_plrn.txt 2>&1 || { tail -20 gpurun_out/al_plrn.txt; exit 4; }
grep -v amdgpu.ids gpurun_out/al_plrn.txt | tail -12
: > gpurun_out/al_bench.jsonl
for m in caffenet googlenet caffenet googlenet; do
  timeout -k 10 300 python -u bench.py --model $m >> gpurun_out/al_bench.jsonl 2> gpurun_out/al_bench.err || { tail -20 gpurun_out/al_bench.err; exit 5; }
  echo "$m: $(tail -1 gpurun_out/al_bench.jsonl | cut -c45-75)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cn7 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_cn7.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_cn7.log; exit 6; }
f=$(ls gpurun_out/prof_cn7/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/prof_cn7/run_kernel_trace.csv)
python3 scripts/prof_summary.py "$f" all > gpurun_out/prof_cn7_summary.txt && head -28 gpurun_out/prof_cn7_summary.txt
rm -rf gpurun_out/prof_cn7
