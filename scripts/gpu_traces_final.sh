# round-6 final kernel traces: one step each of CaffeNet, AlexNet, GoogLeNet and VGG-16 fp8
# (rocprofv3 --kernel-trace, summarised per iteration by scripts/prof_summary.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name, bench args...
  local n=$1; shift
  rm -rf gpurun_out/prof_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run --output-format csv -- python3 bench.py --steps 4 --warmup 3 "$@" > gpurun_out/prof_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/prof_$n.log; return 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_$n all > gpurun_out/prof_${n}_summary.txt 2>&1
  head -12 gpurun_out/prof_${n}_summary.txt
}
run f6caffenet && run f6alexnet --model alexnet && run f6googlenet --model googlenet && run f6vggfp8 --model vgg16 --dtype fp8
rm -rf gpurun_out/prof_f6*/*/ 2>/dev/null; true
