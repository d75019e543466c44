#!/bin/bash
# Round 3 session AP: decode bench with the greedy graph warmed before the timed loop; long-row
# ffn_down stages per quant type at T = 1 (AMDK8S_LLM_LONGROW unset / q4 / q6 / 1), GEMV-level and
# step-level.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ap
mkdir -p $OUT
for lr in def q4 q6 1; do
  if [ $lr = def ]; then unset AMDK8S_LLM_LONGROW; else export AMDK8S_LLM_LONGROW=$lr; fi
  timeout -k 10 300 python -u tools/llm_bench.py --tokens 1,4 --gemv --gemv-cases down_q4k,down_q6k \
    --out $OUT/llm_bench_lr_$lr.json > $OUT/llm_bench_lr_$lr.log 2>&1 || { tail -30 $OUT/llm_bench_lr_$lr.log; exit 1; }
  echo "== LONGROW=$lr"; grep -E "decode T|'cfg': \[0, 0\]" $OUT/llm_bench_lr_$lr.log
done
