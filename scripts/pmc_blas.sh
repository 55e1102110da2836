#!/bin/bash
# rocprofv3 PMC passes over scripts/pmc_blas.py: hipBLASLt vs gemm_kernel on the same products
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmcb
mkdir -p $out
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INST_LEVEL_LDS" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $out/p$i -o run --output-format csv -- python3 scripts/pmc_blas.py > $out/p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 $out/p$i.log; exit 1; }
done
python3 scripts/pmc_agg.py $out --by-grid > $out/summary.txt 2>&1; cat $out/summary.txt
