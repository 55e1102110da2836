set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp32_device_gpu.py > gpurun_out/fp32chk_tests.log 2>&1 && tail -3 gpurun_out/fp32chk_tests.log &&
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 2 > gpurun_out/fp32chk_bench.json 2> gpurun_out/fp32chk_bench.err && cat gpurun_out/fp32chk_bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32 -o run -- python bench.py --dtype fp32 --steps 3 --warmup 1 > gpurun_out/fp32chk_prof.log 2>&1; echo prof rc $?
