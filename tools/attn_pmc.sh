#!/usr/bin/env bash
# PMC passes over the flash-attention kernel at Wan2.1's self-attention shape (2x12 heads, 2560
# tokens, d=128), one QT per run; counters with --kernel-trace only (pool rules).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/attn_pmc}
mkdir -p $OUT
for qt in ${QTS:-1 4}; do
  export ATTN_ONLY=wan_self ATTN_QTS=$qt
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY \
    -d $OUT/qt$qt/p1 -o p1 --output-format csv -- python3 tools/attn_probe.py > $OUT/qt$qt.p1.log 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_ADDR_CONFLICT SQ_CYCLES GRBM_GUI_ACTIVE \
    -d $OUT/qt$qt/p2 -o p2 --output-format csv -- python3 tools/attn_probe.py > $OUT/qt$qt.p2.log 2>&1
done
echo done
