# round 6: kernel trace of one fp32-device-mode CaffeNet step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/prof_fp32
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32 -o run --output-format csv -- python3 bench.py --dtype fp32 --steps 3 --warmup 1 > gpurun_out/prof_fp32.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_fp32.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof_fp32 all > gpurun_out/prof_fp32_summary.txt 2>&1
head -45 gpurun_out/prof_fp32_summary.txt
rm -rf gpurun_out/prof_fp32/*/ 2>/dev/null; true
