#!/bin/bash
# fp8 fidelity-setting sweep (chaos floor bf16 vs bf16alt) + VGG-16 b2048 fp8 kernel trace (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for noise in ${NOISES:-0.5 0.3}; do
  timeout -k 10 300 python -u scripts/fp8_trajectory.py --steps 200 --noise $noise --modes bf16,bf16alt,fp8dgw > gpurun_out/fp8_traj_n$noise.txt 2>&1 || { tail -20 gpurun_out/fp8_traj_n$noise.txt; exit 3; }
  echo "== noise $noise"; grep -v amdgpu.ids gpurun_out/fp8_traj_n$noise.txt
done
rm -rf gpurun_out/prof_vgg8
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vgg8 -o run --output-format csv -- python3 bench.py --model vgg16 --dtype fp8 --steps 4 --warmup 2 > gpurun_out/prof_vgg8.log 2>&1 || { tail -20 gpurun_out/prof_vgg8.log; exit 4; }
python3 scripts/prof_summary.py gpurun_out/prof_vgg8 > gpurun_out/prof_vgg8_summary.txt 2>&1; cat gpurun_out/prof_vgg8_summary.txt
rm -f gpurun_out/prof_vgg8/run_kernel_trace.csv
