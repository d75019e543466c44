#!/bin/bash
# Round 3 session AD: rmsnorm_q8 summing squares in the GEMV prologue's order (bit-identical
# norms, norm-in-prologue only for steps of <= 2 tokens) and the prefill glue kernels
# (llm_prefill.hip) — LLM GPU tests, decode T=1..4 + prefill, prefill steady-state profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ad
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_prefill -o llm -- \
  python3 tools/steady_prof.py llm-prefill --iters 10 --warmup 3 > $OUT/prof_prefill.log 2>&1 \
  || { tail -20 $OUT/prof_prefill.log; exit 1; }
tail -1 $OUT/prof_prefill.log
python3 tools/rocpd_summary.py $(find $OUT/prof_prefill -name '*.db' | head -1) --after-gap-ms 200 \
  --per 10 --top 30 > $OUT/llm_prefill_kernels.txt && head -20 $OUT/llm_prefill_kernels.txt | cut -c1-170
