#!/usr/bin/env bash
# PMC passes over the LLM prompt-attention kernel (llm_prefill_attn.hip) on one shape
# (PROBE_P queries at PROBE_STARTS, default 8192 at 0: the monolithic-prefill case); counters with
# --kernel-trace only (pool rules), one pass per run, each under its own time limit.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prefill_attn_pmc}
mkdir -p "$OUT"
export PROBE_P=${PROBE_P:-8192} PROBE_STARTS=${PROBE_STARTS:-0} PROBE_VARIANTS=hand
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY \
  -d "$OUT/p1" -o p1 --output-format csv -- python3 tools/debug/prefill_attn_probe.py > "$OUT/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_ADDR_CONFLICT SQ_CYCLES GRBM_GUI_ACTIVE \
  -d "$OUT/p2" -o p2 --output-format csv -- python3 tools/debug/prefill_attn_probe.py > "$OUT/p2.log" 2>&1
PMC_MATCH=prefill_attn python3 tools/pmc_summary.py "$OUT/**/*counter_collection.csv"
