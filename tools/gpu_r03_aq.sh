#!/bin/bash
# Round 3 session AQ: Q4_K ffn_down in long-row stages at every T (new default): LLM GPU tests,
# decode bench, ffn_down decomposition sweep at T = 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/aq
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -1 $OUT/pytest_llm.log
timeout -k 10 400 python -u tools/llm_bench.py --gemv --gemv-cases down_q4k,down_q6k \
  --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode T|prefill|'T': 1," $OUT/llm_bench.log | cut -c1-160
