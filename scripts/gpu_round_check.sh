# Round-end style GPU check: gpu tests, smoke, CaffeNet + GoogLeNet benches, kernel profile.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 && tail -2 gpurun_out/gpu_tests.log && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 python -u bench.py > gpurun_out/c.json 2> gpurun_out/c.err && cat gpurun_out/c.json && \
timeout -k 10 240 python -u bench.py --model googlenet --steps 30 --warmup 5 > gpurun_out/g.json 2> gpurun_out/g.err && \
cat gpurun_out/g.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > gpurun_out/prof.log 2>&1 && echo PROF_OK
