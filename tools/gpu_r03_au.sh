#!/bin/bash
# Round 3 session AU: prefill q stored token-major for SDPA (AMDK8S_LLM_PREFILL_QTOK) — SDPA layout
# probe, LLM GPU tests, prefill timing with the knob on / off.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/au
mkdir -p $OUT
timeout -k 10 200 python -u tools/debug/sdpa_layout_probe.py > $OUT/sdpa_layout_probe.log 2>&1 \
  || { tail -30 $OUT/sdpa_layout_probe.log; exit 1; }
cat $OUT/sdpa_layout_probe.log
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -1 $OUT/pytest_llm.log
for q in 1 0 1 0; do
  AMDK8S_LLM_PREFILL_QTOK=$q timeout -k 10 300 python -u tools/llm_bench.py --tokens 1 --steps 32 \
    --out $OUT/llm_bench_q$q.json > $OUT/llm_bench_q$q.log 2>&1 || { tail -30 $OUT/llm_bench_q$q.log; exit 1; }
  echo "QTOK=$q $(grep prefill $OUT/llm_bench_q$q.log | grep -v '^{')"
done
