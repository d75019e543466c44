#!/bin/bash
# Round 3 session P: LLM decode with two balanced stages per ffn_down row (AMDK8S_LLM_LONGROW A/B),
# GEMV sweep, tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
for lr in 0 1; do
  AMDK8S_LLM_LONGROW=$lr timeout -k 10 400 python -u tools/llm_bench.py --gemv --out $OUT/llm_bench_lr$lr.json \
    > $OUT/llm_bench_lr$lr.log 2>&1 || { tail -30 $OUT/llm_bench_lr$lr.log; exit 1; }
  echo "longrow=$lr"; grep -v '^{' $OUT/llm_bench_lr$lr.log | grep -E "decode|prefill"
done
