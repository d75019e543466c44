#!/usr/bin/env bash
# PMC passes for GEMM arms (counters only with --kernel-trace, per pool rules).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SHAPE=${SHAPE:-8192x8192x8192}
for arm in ${ARMS:-w8 w4 blt}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc/$arm/p1 -o p1 --output-format csv -- python3 tools/gemm_arm.py --arm $arm --shape $SHAPE --iters 10 > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE \
    -d gpurun_out/pmc/$arm/p2 -o p2 --output-format csv -- python3 tools/gemm_arm.py --arm $arm --shape $SHAPE --iters 10 > /dev/null 2>&1
  echo "== $arm"; python3 tools/pmc_summary.py "gpurun_out/pmc/$arm/**/*counter_collection.csv"
done
