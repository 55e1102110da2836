# round 6: tuning-DB coverage / reproducibility tests, then the zoo benches on the final DB
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tune_db_gpu.py > gpurun_out/r6k_tunedb.log 2>&1; rc=$?; echo "tune-db tests rc $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r6k_tunedb.log | tail -9
case $rc in 0|1) ;; *) exit $rc;; esac
: > gpurun_out/r6k_bench.jsonl
b() { timeout -k 10 300 python bench.py "$@" >> gpurun_out/r6k_bench.jsonl 2>> gpurun_out/r6k_bench.err || { echo "bench $* failed"; tail -5 gpurun_out/r6k_bench.err; exit 1; }; tail -1 gpurun_out/r6k_bench.jsonl | cut -c1-160; }
b && b && b --model googlenet && b --model googlenet && b --model vgg16 && b --model vgg16 --dtype fp8 && b --model alexnet && b --dtype fp32 --steps 10 --warmup 2
