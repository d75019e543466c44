#!/bin/bash
# Round 3 session AF: the attention combine inside the o_proj GEMV prologue (qgemv_attn) — LLM GPU
# tests, decode A/B over AMDK8S_LLM_ATTN_PROLOGUE and the o_proj decomposition, T=1 profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/af
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
for cfg in "0 8,16" "1 8,16" "1 8,8" "1 4,8"; do
  set -- $cfg
  AMDK8S_LLM_ATTN_PROLOGUE=$1 AMDK8S_LLM_ATTN_OPROJ=$2 timeout -k 10 300 python -u tools/llm_bench.py \
    --out $OUT/llm_bench_ap$1_$2.json > $OUT/llm_bench_ap$1_$2.log 2>&1 || { tail -30 $OUT/llm_bench_ap$1_$2.log; exit 1; }
  echo "attn_prologue=$1 oproj=$2"; grep -E "decode" $OUT/llm_bench_ap$1_$2.log | grep -v '^{'
done
AMDK8S_LLM_ATTN_PROLOGUE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t1 -o llm -- \
  python3 tools/steady_prof.py llm-decode --tokens 1 --iters 64 --warmup 8 > $OUT/prof_t1.log 2>&1 \
  || { tail -20 $OUT/prof_t1.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_t1 -name '*.db' | head -1) --after-gap-ms 200 \
  --per 64 --top 30 > $OUT/llm_decode_t1_kernels.txt && head -14 $OUT/llm_decode_t1_kernels.txt | cut -c1-150
