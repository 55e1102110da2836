#!/bin/bash
# rocprofv3 kernel traces of one training step: CaffeNet (headline), VGG-16 b2048 fp8, GoogLeNet b128 (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
run() {  # name, bench args...
  local n=$1; shift
  rm -rf gpurun_out/prof_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 "$@" > gpurun_out/prof_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/prof_$n.log; return 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_$n > gpurun_out/prof_${n}_summary.txt 2>&1
  head -30 gpurun_out/prof_${n}_summary.txt
}
run caffenet && run googlenet --model googlenet && run vgg16fp8 --model vgg16 --dtype fp8
