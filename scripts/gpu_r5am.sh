#!/bin/bash
# GoogLeNet conv2/3x3 (M=401408, N=192, K=576) and CaffeNet conv3: implicit conv vs dense GEMM of equal shape, every tile
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/conv_probe.py --case gn_conv2,gn_3b_3x3,cn_conv3 > gpurun_out/am_conv.txt 2>&1 || { tail -20 gpurun_out/am_conv.txt; exit 4; }
grep -v amdgpu.ids gpurun_out/am_conv.txt
