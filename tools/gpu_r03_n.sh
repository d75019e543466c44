#!/bin/bash
# Round 3 session N: LLM decode with the chunk merge inside the attention kernel (last-arriving
# workgroup) — tests (bit-identical to the combine kernel, counters stay zero), bench A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/n
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
for fc in 0 1; do
  AMDK8S_LLM_FUSED_COMBINE=$fc timeout -k 10 400 python -u tools/llm_bench.py --kernels --out $OUT/llm_bench_fc$fc.json \
    > $OUT/llm_bench_fc$fc.log 2>&1 || { tail -30 $OUT/llm_bench_fc$fc.log; exit 1; }
  echo "fused_combine=$fc"; grep -v '^{' $OUT/llm_bench_fc$fc.log | grep -E "decode|prefill"
done
