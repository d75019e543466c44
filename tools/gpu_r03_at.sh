#!/bin/bash
# Round 3 session AT: 3-deep weight ring for one-stage GEMV rows (gate|up pair walks 8 rows per
# wave) — LLM GPU tests, decode bench, T = 1 / T = 2 steady-state kernel profiles.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/at
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -1 $OUT/pytest_llm.log
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
for T in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t$T -o llm -- \
    python3 tools/steady_prof.py llm-decode --tokens $T --iters 64 --warmup 8 > $OUT/prof_t$T.log 2>&1 \
    || { tail -20 $OUT/prof_t$T.log; exit 1; }
  python3 tools/rocpd_summary.py $(find $OUT/prof_t$T -name '*.db' | head -1) --after-gap-ms 200 \
    --per 64 --top 30 > $OUT/llm_decode_t${T}_kernels.txt && head -5 $OUT/llm_decode_t${T}_kernels.txt | cut -c1-120 \
    && grep "1, 0, 2, true\|2, 0, 2, true" $OUT/llm_decode_t${T}_kernels.txt | cut -c1-120
done
