#!/bin/bash
# average VMEM / LDS instruction latency of the conv GEMM (level / count counters)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmcl_${CASE:-fwd}
mkdir -p $out
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $out/p1 -o run --output-format csv -- python3 scripts/pmc_conv.py > $out/p1.log 2>&1 || { echo "pmc failed"; tail -5 $out/p1.log; exit 1; }
python3 scripts/pmc_agg.py $out
