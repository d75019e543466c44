#!/bin/bash
# Round 3 session Q: attention reverted (probe + Wan / SD benches back to the round-3 numbers?),
# LLM decode A/B: long-row balanced stages, gate|up → Q8 epilogue; LLM tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/q
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
for cfg in "0 0" "1 0" "1 1"; do
  set -- $cfg
  AMDK8S_LLM_LONGROW=$1 AMDK8S_LLM_PAIR_Q8=$2 timeout -k 10 400 python -u tools/llm_bench.py \
    --out $OUT/llm_bench_lr$1_pq$2.json > $OUT/llm_bench_lr$1_pq$2.log 2>&1 || { tail -30 $OUT/llm_bench_lr$1_pq$2.log; exit 1; }
  echo "longrow=$1 pair_q8=$2"; grep -v '^{' $OUT/llm_bench_lr$1_pq$2.log | grep -E "decode"
done
ATTN_VARIANTS=2 timeout -k 10 300 python -u tools/attn_probe.py > $OUT/attn_probe.log 2>&1 || { tail -20 $OUT/attn_probe.log; exit 1; }
grep -E "wan_self|sd_64" $OUT/attn_probe.log | grep -v '^{'
timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560.json > $OUT/wan_bench_2560.log 2>&1 || { tail -20 $OUT/wan_bench_2560.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560.log
