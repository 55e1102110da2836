#!/bin/bash
# one gpurun call: pool+LRN tile probe, full GPU suite, CaffeNet bench x2 + step trace, VGG-16 b2048 fp8 vs bf16
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 180 python3 scripts/plrn_probe.py "20000,32768,48000" 4,8 > gpurun_out/plrn_probe2.txt 2>&1 || { grep -v amdgpu.ids gpurun_out/plrn_probe2.txt | tail -20; exit 3; }
grep -v amdgpu.ids gpurun_out/plrn_probe2.txt | grep -E "forward|mask_lds . budget 32768 cg None|reference"
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc, stopping"; exit $rc; fi
: > gpurun_out/bench_round.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py >> gpurun_out/bench_round.jsonl 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 5; }
  tail -1 gpurun_out/bench_round.jsonl | cut -c1-200
done
rm -rf gpurun_out/prof_caffenet
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_caffenet -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 > gpurun_out/prof_caffenet.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_caffenet.log; exit 6; }
python3 scripts/prof_summary.py gpurun_out/prof_caffenet > gpurun_out/prof_caffenet_summary.txt 2>&1; tail -1 gpurun_out/prof_caffenet_summary.txt
: > gpurun_out/vgg_final.jsonl
for dt in fp8 bf16; do
  timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 --dtype $dt >> gpurun_out/vgg_final.jsonl 2> gpurun_out/vgg_final.err || { echo "vgg $dt failed"; tail -5 gpurun_out/vgg_final.err; exit 4; }
  tail -1 gpurun_out/vgg_final.jsonl | cut -c1-180
done
exit $rc
