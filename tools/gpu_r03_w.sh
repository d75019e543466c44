#!/bin/bash
# Round 3 session W: the LLM decode GPU tests (fused residual norm tail, single-pass multi-head
# attention merge, two-matrix q|k|v GEMV), decode A/B over AMDK8S_LLM_RESID_NORM x
# AMDK8S_LLM_FUSED_COMBINE x AMDK8S_LLM_QKV2, and
# steady-state T=1 kernel profiles of the default and the fully fused step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/w
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
for cfg in "0 0 0" "0 0 1" "1 0 1" "0 1 1" "1 1 1"; do
  set -- $cfg
  AMDK8S_LLM_RESID_NORM=$1 AMDK8S_LLM_FUSED_COMBINE=$2 AMDK8S_LLM_QKV2=$3 timeout -k 10 300 python -u tools/llm_bench.py \
    --out $OUT/llm_bench_rn$1_fc$2_q$3.json > $OUT/llm_bench_rn$1_fc$2_q$3.log 2>&1 || { tail -30 $OUT/llm_bench_rn$1_fc$2_q$3.log; exit 1; }
  echo "resid_norm=$1 fused_combine=$2 qkv2=$3"; grep -v '^{' $OUT/llm_bench_rn$1_fc$2_q$3.log | grep -E "decode"
done
for cfg in "0 0" "1 1"; do
  set -- $cfg
  AMDK8S_LLM_QKV2=$2 AMDK8S_LLM_RESID_NORM=$1 AMDK8S_LLM_FUSED_COMBINE=$2 timeout -k 10 300 rocprofv3 --kernel-trace \
    --output-format rocpd -d $OUT/prof_rn$1_fc$2 -o llm -- \
    python3 tools/steady_prof.py llm-decode --tokens 1 --iters 64 --warmup 8 > $OUT/prof_rn$1_fc$2.log 2>&1 \
    || { tail -20 $OUT/prof_rn$1_fc$2.log; exit 1; }
  tail -1 $OUT/prof_rn$1_fc$2.log
  python3 tools/rocpd_summary.py $(find $OUT/prof_rn$1_fc$2 -name '*.db' | head -1) --after-gap-ms 200 \
    --per 64 --top 30 > $OUT/llm_decode_t1_rn$1_fc$2_kernels.txt && head -16 $OUT/llm_decode_t1_rn$1_fc$2_kernels.txt | cut -c1-150
done
