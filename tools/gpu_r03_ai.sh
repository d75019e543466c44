#!/bin/bash
# Round 3 session AI: the prefill GEMMs at M = 512 on every gemm_epi path vs hipBLASLt, plus the
# LLM GPU tests and decode with the long-row stages from T = 3 and the GQA prefill on by default.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ai
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
timeout -k 10 400 python -u tools/llm_prefill_gemm_probe.py --m 512 --out $OUT/prefill_gemm_probe.json \
  > $OUT/prefill_gemm_probe.log 2>&1 || { tail -30 $OUT/prefill_gemm_probe.log; exit 1; }
grep -E "auto|torch" $OUT/prefill_gemm_probe.log | cut -c1-160
