#!/bin/bash
# Round 3 session L: LLM decode with the GEMV inputs quantised once per step (rmsnorm_q8) instead
# of in every GEMV workgroup's prologue — A/B over T = 1..4, tests with the split path.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/l
mkdir -p $OUT
for q in 0 1; do
  AMDK8S_LLM_Q8SPLIT=$q timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench_q8split$q.json \
    > $OUT/llm_bench_q8split$q.log 2>&1 || { tail -30 $OUT/llm_bench_q8split$q.log; exit 1; }
  echo "q8split=$q"; grep -v '^{' $OUT/llm_bench_q8split$q.log | grep -E "decode|prefill"
done
AMDK8S_LLM_Q8SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm_q8split.log 2>&1 || { tail -60 $OUT/pytest_llm_q8split.log; exit 1; }
tail -2 $OUT/pytest_llm_q8split.log
