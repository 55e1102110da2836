# round 6: fp32 device mode check (split-K), pool+LRN backward forms, fp8 gate + trajectories
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_device_gpu.py > gpurun_out/fp32chk_tests.log 2>&1 || { tail -30 gpurun_out/fp32chk_tests.log; exit 1; }
tail -2 gpurun_out/fp32chk_tests.log
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 2 > gpurun_out/fp32chk_bench.json 2> gpurun_out/fp32chk_bench.err || { tail gpurun_out/fp32chk_bench.err; exit 1; }
cut -c1-200 gpurun_out/fp32chk_bench.json
bash scripts/archive/gpu_r6d.sh
