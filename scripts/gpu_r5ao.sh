#!/bin/bash
# persistent ring-pipelined tiles (gemm_pk.h) vs the tuned tile on GoogLeNet's small-K 3x3 convs
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/conv_probe.py --case gn_conv2,gn_3b_3x3 --tiles=-1,15,17,10,30,31,32,33,34,36,37,38,40,41 --no-dense > gpurun_out/ao_conv.txt 2>&1 || { tail -20 gpurun_out/ao_conv.txt; exit 4; }
grep -v amdgpu.ids gpurun_out/ao_conv.txt
