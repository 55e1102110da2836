#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/direct8_probe.py 256 > gpurun_out/direct8_probe.txt 2>&1; rc=$?; cat gpurun_out/direct8_probe.txt; [ $rc -eq 0 ] || exit $rc
SN_CONV_DIRECT_FP8=0 timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 --dtype fp8 > gpurun_out/vgg_nodirect.json 2> gpurun_out/vgg_nodirect.err || { tail -5 gpurun_out/vgg_nodirect.err; exit 4; }
cut -c1-200 gpurun_out/vgg_nodirect.json
TILES=0 WGRAD_TILES=0 bash scripts/pmc_tiles.sh > gpurun_out/ab_pmc.log 2>&1 || { tail -20 gpurun_out/ab_pmc.log; exit 6; }
tail -12 gpurun_out/ab_pmc.log
