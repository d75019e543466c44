#!/bin/bash
# Round 3 session AH: re-measure the older GEMV A/B knobs on the current kernels — register-resident
# activations up to T=4 (AMDK8S_LLM_REGX_T=4) and two balanced stages for the 74-block ffn_down
# rows (AMDK8S_LLM_LONGROW=1).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ah
mkdir -p $OUT
for cfg in "2 0" "4 0" "2 1" "4 1"; do
  set -- $cfg
  AMDK8S_LLM_REGX_T=$1 AMDK8S_LLM_LONGROW=$2 timeout -k 10 300 python -u tools/llm_bench.py --steps 96 \
    --out $OUT/llm_bench_rx$1_lr$2.json > $OUT/llm_bench_rx$1_lr$2.log 2>&1 || { tail -30 $OUT/llm_bench_rx$1_lr$2.log; exit 1; }
  echo "regx_t=$1 longrow=$2"; grep -E "decode" $OUT/llm_bench_rx$1_lr$2.log | grep -v '^{'
done
