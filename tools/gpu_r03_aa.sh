#!/bin/bash
# Round 3 session AA: MFMA decode attention (one workgroup per 1024 positions, no combine launch)
# and the attn/ffn RMSNorm inside the GEMV prologues — LLM GPU tests, decode A/B over
# AMDK8S_LLM_ATTN x AMDK8S_LLM_NORM_PROLOGUE, T=1 / T=4 steady-state profiles of the default.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
for cfg in "split 0" "mfma 0" "mfma 1" "split 1"; do
  set -- $cfg
  AMDK8S_LLM_ATTN=$1 AMDK8S_LLM_NORM_PROLOGUE=$2 timeout -k 10 300 python -u tools/llm_bench.py \
    --out $OUT/llm_bench_$1_np$2.json > $OUT/llm_bench_$1_np$2.log 2>&1 || { tail -30 $OUT/llm_bench_$1_np$2.log; exit 1; }
  echo "attn=$1 norm_prologue=$2"; grep -E "decode" $OUT/llm_bench_$1_np$2.log | grep -v '^{'
done
for T in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t$T -o llm -- \
    python3 tools/steady_prof.py llm-decode --tokens $T --iters 64 --warmup 8 > $OUT/prof_t$T.log 2>&1 \
    || { tail -20 $OUT/prof_t$T.log; exit 1; }
  python3 tools/rocpd_summary.py $(find $OUT/prof_t$T -name '*.db' | head -1) --after-gap-ms 200 \
    --per 64 --top 30 > $OUT/llm_decode_t${T}_kernels.txt && head -14 $OUT/llm_decode_t${T}_kernels.txt | cut -c1-150
done
