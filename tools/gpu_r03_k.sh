#!/bin/bash
# Round 3 session K: split-K with the gated residual in the finalize pass (tests), LLM decode with
# the Infinity-Cache prefetch of gate|up on a side stream (A/B over prefetch workgroups), prefill.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/k
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -2 $OUT/gemm_epi_tests.log
for pf in 0 32 96; do
  AMDK8S_LLM_PREFETCH=$pf timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench_pf$pf.json \
    > $OUT/llm_bench_pf$pf.log 2>&1 || { tail -30 $OUT/llm_bench_pf$pf.log; exit 1; }
  echo "prefetch wgs=$pf"; grep -v '^{' $OUT/llm_bench_pf$pf.log | grep -E "decode|prefill"
done
AMDK8S_LLM_PREFETCH=32 timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm_pf.log 2>&1 || { tail -60 $OUT/pytest_llm_pf.log; exit 1; }
tail -2 $OUT/pytest_llm_pf.log
