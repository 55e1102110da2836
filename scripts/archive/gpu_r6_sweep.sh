# round 6: wider split-K sweeps of the CaffeNet weight gradients and the InnerProduct products
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/wgrad_probe.py --case conv1f --tiles 0,10,1,13,21,22 --splits 27,54,81,109,160,218 --forms implicit > gpurun_out/sw_conv1.txt 2>&1 || { tail -20 gpurun_out/sw_conv1.txt; exit 1; }
grep -v amdgpu gpurun_out/sw_conv1.txt
timeout -k 10 400 python -u scripts/wgrad_probe.py --case conv2,conv3,conv5 --tiles 0,10,1,13,16 --splits 8,12,16,20,25,32 --forms implicit > gpurun_out/sw_conv.txt 2>&1 || { tail -20 gpurun_out/sw_conv.txt; exit 1; }
grep -v amdgpu gpurun_out/sw_conv.txt
timeout -k 10 400 python -u scripts/fc_probe.py > gpurun_out/sw_fc.txt 2>&1 || { tail -20 gpurun_out/sw_fc.txt; exit 1; }
grep -v amdgpu gpurun_out/sw_fc.txt | tail -30
