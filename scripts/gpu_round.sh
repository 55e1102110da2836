#!/bin/bash
# one gpurun call: full GPU suite, then CaffeNet bench and VGG-16 b2048 fp8 vs bf16 on the same box
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -12 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc, stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 5; }
cut -c1-200 gpurun_out/bench.json
: > gpurun_out/vgg_final.jsonl
for dt in fp8 bf16; do
  timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 --dtype $dt >> gpurun_out/vgg_final.jsonl 2> gpurun_out/vgg_final.err || { echo "vgg $dt failed"; tail -5 gpurun_out/vgg_final.err; exit 4; }
  tail -1 gpurun_out/vgg_final.jsonl | cut -c1-180
done
exit $rc
