#!/bin/bash
# Round 3 session AC: steady-state kernel profile of the 512-token LLM prompt prefill (fp16 dense
# path on the hand-written GEMMs) — where time-to-first-token goes.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ac
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_prefill -o llm -- \
  python3 tools/steady_prof.py llm-prefill --iters 10 --warmup 3 > $OUT/prof_prefill.log 2>&1 \
  || { tail -20 $OUT/prof_prefill.log; exit 1; }
tail -1 $OUT/prof_prefill.log
python3 tools/rocpd_summary.py $(find $OUT/prof_prefill -name '*.db' | head -1) --after-gap-ms 200 \
  --per 10 --top 40 > $OUT/llm_prefill_kernels.txt && head -30 $OUT/llm_prefill_kernels.txt | cut -c1-170
