#!/bin/bash
# Round 3 session AS: waves per gate|up (pair -> Q8) workgroup of 32 rows (AMDK8S_LLM_PAIR_WAVES
# unset = 4, 8, 2) at T = 1..4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/as
mkdir -p $OUT
for pw in def 8 2; do
  if [ $pw = def ]; then unset AMDK8S_LLM_PAIR_WAVES; else export AMDK8S_LLM_PAIR_WAVES=$pw; fi
  timeout -k 10 300 python -u tools/llm_bench.py --out $OUT/llm_bench_pw_$pw.json > $OUT/llm_bench_pw_$pw.log 2>&1 \
    || { tail -30 $OUT/llm_bench_pw_$pw.log; exit 1; }
  echo "== PAIR_WAVES=$pw"; grep -E "decode T" $OUT/llm_bench_pw_$pw.log
done
