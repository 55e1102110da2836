#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
rm -rf gpurun_out/pmcn && mkdir -p gpurun_out/pmcn
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcn/p1 -o run --output-format csv -- python3 scripts/newk_probe.py > gpurun_out/pmcn/p1.log 2>&1 || { tail -5 gpurun_out/pmcn/p1.log; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmcn/p2 -o run --output-format csv -- python3 scripts/newk_probe.py > gpurun_out/pmcn/p2.log 2>&1 || { tail -5 gpurun_out/pmcn/p2.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcn/p3 -o run --output-format csv -- python3 scripts/newk_probe.py > gpurun_out/pmcn/p3.log 2>&1 || { tail -5 gpurun_out/pmcn/p3.log; exit 5; }
find gpurun_out/pmcn -name "*counter_collection.csv" | head
for d in p1 p2 p3; do f=$(find gpurun_out/pmcn/$d -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/pmcn/$d/run_counter_collection.csv; done
python3 scripts/pmc_newk_agg.py gpurun_out/pmcn | tee gpurun_out/pmc_newk.txt
