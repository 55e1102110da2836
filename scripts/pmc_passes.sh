#!/bin/bash
# rocprofv3 PMC passes over scripts/pmc_gemm.py (one counter group per run; program directly after --)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
PROG=${PROG:-scripts/pmc_gemm.py}
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc/list_avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 $PROG $PROG_ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok"
done
