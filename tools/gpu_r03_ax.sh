#!/bin/bash
# Round 3 session AX: re-measure the attn/ffn RMSNorm in the GEMV prologues at T = 3 / 4
# (AMDK8S_LLM_NORM_PROLOGUE_T = 2 default vs 4) on the round's final kernels, alternating runs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ax
mkdir -p $OUT
for r in a b; do
  for pt in 2 4; do
    AMDK8S_LLM_NORM_PROLOGUE_T=$pt timeout -k 10 300 python -u tools/llm_bench.py --tokens 3,4 \
      --out $OUT/llm_bench_pt${pt}_$r.json > $OUT/llm_bench_pt${pt}_$r.log 2>&1 || { tail -30 $OUT/llm_bench_pt${pt}_$r.log; exit 1; }
    echo "== NORM_PROLOGUE_T=$pt ($r)"; grep -E "decode T" $OUT/llm_bench_pt${pt}_$r.log
  done
done
