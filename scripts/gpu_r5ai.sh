#!/bin/bash
# GoogLeNet max-pool shapes in isolation (b128): timing, then HBM / L2 / L1 counters per kernel
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "pool" > gpurun_out/ai_tests.log 2>&1 || { tail -40 gpurun_out/ai_tests.log; exit 3; }
tail -1 gpurun_out/ai_tests.log
timeout -k 10 300 python -u scripts/pool_probe.py --batch 128 --only "gn" > gpurun_out/ai_probe.txt 2>&1 || { tail -20 gpurun_out/ai_probe.txt; exit 4; }
cat gpurun_out/ai_probe.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_pool/pA -o run --output-format csv -- python3 scripts/pool_probe.py --batch 128 --only "gn 3a,gn 4a" --reps 2 > gpurun_out/ai_pA.log 2>&1 || { tail -5 gpurun_out/ai_pA.log; exit 5; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_pool/pB -o run --output-format csv -- python3 scripts/pool_probe.py --batch 128 --only "gn 3a,gn 4a" --reps 2 > gpurun_out/ai_pB.log 2>&1 || { tail -5 gpurun_out/ai_pB.log; exit 6; }
python3 scripts/pmc_kernels.py gpurun_out/pmc_pool/pA gpurun_out/pmc_pool/pB --match pool > gpurun_out/ai_pmc.txt && cat gpurun_out/ai_pmc.txt
rm -rf gpurun_out/pmc_pool
