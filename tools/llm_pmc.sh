#!/usr/bin/env bash
# PMC passes over a short Qwen2.5-7B-shaped decode (tools/llm_bench.py), counters only with
# --kernel-trace (pool rules).  Summary per kernel: duration, wait / busy shares,
# HBM read bytes.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/llm_pmc}
TOKENS=${TOKENS:-1}
CMD="python3 tools/llm_bench.py --layers 4 --steps 24 --tokens $TOKENS --prompt 128"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
  -d $OUT/p1 -o p1 --output-format csv -- $CMD > $OUT.p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  -d $OUT/p2 -o p2 --output-format csv -- $CMD > $OUT.p2.log 2>&1
python3 tools/llm_pmc_summary.py "$OUT/**/*counter_collection.csv"
