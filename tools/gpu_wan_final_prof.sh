#!/usr/bin/env bash
# Final Wan evidence: rocprofv3 kernel stats of the DiT step (HIP-graph arm) and a PMC pass over the
# transposed-score attention kernel at the Wan self-attention shape.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT="${OUT:-gpurun_out/wanprof}"
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/step" -o step --output-format csv -- python3 tools/wan_bench.py --arms native --iters 4 --warmup 1 --no-e2e > "$OUT/step.log" 2>&1
ATTN_ONLY=wan_self ATTN_QTS=4 ATTN_VARIANTS=0 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY \
  -d "$OUT/attn/p1" -o p1 --output-format csv -- python3 tools/attn_probe.py > "$OUT/attn_p1.log" 2>&1
ATTN_ONLY=wan_self ATTN_QTS=4 ATTN_VARIANTS=0 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_ADDR_CONFLICT SQ_CYCLES GRBM_GUI_ACTIVE \
  -d "$OUT/attn/p2" -o p2 --output-format csv -- python3 tools/attn_probe.py > "$OUT/attn_p2.log" 2>&1
echo done
