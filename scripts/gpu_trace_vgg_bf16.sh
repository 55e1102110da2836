set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/prof_f6vggbf16
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f6vggbf16 -o run --output-format csv -- python3 bench.py --model vgg16 --steps 3 --warmup 2 > gpurun_out/prof_f6vggbf16.log 2>&1 || { tail -5 gpurun_out/prof_f6vggbf16.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof_f6vggbf16 all > gpurun_out/prof_f6vggbf16_summary.txt 2>&1
head -24 gpurun_out/prof_f6vggbf16_summary.txt
rm -rf gpurun_out/prof_f6vggbf16/*/ 2>/dev/null; true
