#!/bin/bash
# Round 3 session Z: rmsnorm_q8 with every load issued up front (one round trip) and DPP quad
# reductions; ffn_down 16 rows per workgroup from T = 3 — LLM GPU tests, decode T=1..4, T=1 / T=4
# steady-state kernel profiles.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/z
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log
for T in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t$T -o llm -- \
    python3 tools/steady_prof.py llm-decode --tokens $T --iters 64 --warmup 8 > $OUT/prof_t$T.log 2>&1 \
    || { tail -20 $OUT/prof_t$T.log; exit 1; }
  python3 tools/rocpd_summary.py $(find $OUT/prof_t$T -name '*.db' | head -1) --after-gap-ms 200 \
    --per 64 --top 30 > $OUT/llm_decode_t${T}_kernels.txt && head -14 $OUT/llm_decode_t${T}_kernels.txt | cut -c1-150
done
