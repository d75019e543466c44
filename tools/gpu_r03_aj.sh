#!/bin/bash
# Round 3 session AJ: Wan2.1 end-to-end job (umT5 encode + 25 steps + VAE decode) and the 14B DiT
# CFG step with the round-3 kernels (the session-U script), then an LLM A/B of the prologue-norm
# step-size threshold (AMDK8S_LLM_NORM_PROLOGUE_T 1 / 2) and long-row stages at T = 2.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/aj
mkdir -p $OUT
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --t5 \
  --out $OUT/wan_bench_e2e.json > $OUT/wan_bench_e2e.log 2>&1 || { tail -20 $OUT/wan_bench_e2e.log; exit 1; }
grep '\[wan_bench\]' $OUT/wan_bench_e2e.log | tail -8
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --no-e2e --model 14b --iters 5 --warmup 2 \
  --out $OUT/wan14b_step.json > $OUT/wan14b_step.log 2>&1 || { tail -20 $OUT/wan14b_step.log; exit 1; }
grep '\[wan_bench\]' $OUT/wan14b_step.log | tail -3
for cfg in "1 -" "2 1"; do
  set -- $cfg
  if [ "$2" = "-" ]; then unset AMDK8S_LLM_LONGROW; else export AMDK8S_LLM_LONGROW=$2; fi
  AMDK8S_LLM_NORM_PROLOGUE_T=$1 timeout -k 10 300 python -u tools/llm_bench.py --tokens 1,2,3 --steps 96 \
    --out $OUT/llm_bench_npt$1_lr$2.json > $OUT/llm_bench_npt$1_lr$2.log 2>&1 || { tail -30 $OUT/llm_bench_npt$1_lr$2.log; exit 1; }
  echo "norm_prologue_T=$1 longrow=$2"; grep -E "decode" $OUT/llm_bench_npt$1_lr$2.log | grep -v '^{'
done
unset AMDK8S_LLM_LONGROW
timeout -k 10 300 python -u tools/llm_bench.py --tokens 1,2,3 --steps 96 --out $OUT/llm_bench_default.json \
  > $OUT/llm_bench_default.log 2>&1 || { tail -30 $OUT/llm_bench_default.log; exit 1; }
echo "defaults"; grep -E "decode" $OUT/llm_bench_default.log | grep -v '^{'
