#!/usr/bin/env bash
# Two PMC passes per GEMM arm on issue/FIFO-stall counters (counters only with --kernel-trace).
# ARMS: space-separated arms of tools/gemm_arm.py (e.g. "w4@AMDK8S_W4_SCHEDULE=l blt").
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SHAPE=${SHAPE:-8192x8192x8192}
for arm in ${ARMS:-w4 blt}; do
  d=gpurun_out/pmc2/$(echo "$arm" | tr '@=' '__')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $d/p1 -o p1 --output-format csv -- python3 tools/gemm_arm.py --arm "$arm" --shape $SHAPE --iters 10 > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $d/p2 -o p2 --output-format csv -- python3 tools/gemm_arm.py --arm "$arm" --shape $SHAPE --iters 10 > /dev/null 2>&1
  echo "== $arm"; python3 tools/pmc_summary.py "$d/**/*counter_collection.csv"
done
