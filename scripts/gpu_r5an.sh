#!/bin/bash
# PMC of GoogLeNet conv2/3x3 forward (small K = 576) on tiles 15 / 10 / 17 vs CaffeNet conv3 (K = 2304) on tile 0
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
rm -rf gpurun_out/pmcc && mkdir -p gpurun_out/pmcc
P="python3 scripts/conv_probe.py --case gn_conv2,cn_conv3 --tiles 15,10,17,0 --reps 2 --no-dense"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcc/p1 -o run --output-format csv -- $P > gpurun_out/pmcc/p1.log 2>&1 || { tail -5 gpurun_out/pmcc/p1.log; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmcc/p2 -o run --output-format csv -- $P > gpurun_out/pmcc/p2.log 2>&1 || { tail -5 gpurun_out/pmcc/p2.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/pmcc/p3 -o run --output-format csv -- $P > gpurun_out/pmcc/p3.log 2>&1 || { tail -5 gpurun_out/pmcc/p3.log; exit 5; }
python3 scripts/pmc_kernels.py gpurun_out/pmcc/p1 gpurun_out/pmcc/p2 gpurun_out/pmcc/p3 --match gemm > gpurun_out/pmc_conv2.txt; cat gpurun_out/pmc_conv2.txt
grep -v amdgpu gpurun_out/pmcc/p1.log | tail -3
rm -rf gpurun_out/pmcc
