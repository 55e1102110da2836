#!/bin/bash
# HIP runtime knobs A/B: device-memory kernel arguments, hardware queues per process
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/envab.txt
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  local v
  v=$(env "${envs[@]}" timeout -k 10 300 python -u bench.py "$@" 2>>gpurun_out/envab.err | grep -o '"value": [0-9.]*') || { echo "$label failed"; tail -5 gpurun_out/envab.err; exit 3; }
  echo "$label $v" | tee -a gpurun_out/envab.txt
}
for i in 1 2; do
  run "caffenet default" X=1 --
  run "caffenet devkernarg" HIP_FORCE_DEV_KERNARG=1 --
done
for i in 1 2; do
  run "googlenet default" X=1 -- --model googlenet
  run "googlenet queues8" GPU_MAX_HW_QUEUES=8 -- --model googlenet
  run "googlenet queues16" GPU_MAX_HW_QUEUES=16 -- --model googlenet
  run "googlenet devkernarg" HIP_FORCE_DEV_KERNARG=1 -- --model googlenet
done
