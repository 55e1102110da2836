#!/bin/bash
# round-5 final evidence: full GPU suite, then the four headline benches (CaffeNet x2, GoogLeNet x2, VGG-16 bf16 / fp8)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 900 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; tail -12 gpurun_out/gpu_tests_final.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc, stopping"; exit $rc; fi
: > gpurun_out/bench_final.jsonl
for m in caffenet googlenet caffenet googlenet; do
  timeout -k 10 300 python -u bench.py --model $m >> gpurun_out/bench_final.jsonl 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 5; }
done
for dt in bf16 fp8; do
  timeout -k 10 500 python -u bench.py --model vgg16 --dtype $dt --steps 6 --warmup 3 >> gpurun_out/bench_final.jsonl 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 6; }
done
grep -o '"model": "[a-z0-9]*"\|"value": [0-9.]*\|"dtype": "[a-z0-9]*"' gpurun_out/bench_final.jsonl | paste - - -
exit $rc
