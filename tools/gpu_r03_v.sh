#!/bin/bash
# Round 3 session V (re-entry after a container reset): the driver's round-end checks on the
# current tree — every GPU test, smoke(), bench.py (1 GPU) — then the LLM decode with the in-launch
# write-through attention combine off / on (AMDK8S_LLM_FUSED_COMBINE).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/v
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-400
for fc in 0 1; do
  AMDK8S_LLM_FUSED_COMBINE=$fc timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench_fc$fc.json \
    > $OUT/llm_bench_fc$fc.log 2>&1 || { tail -30 $OUT/llm_bench_fc$fc.log; exit 1; }
  echo "fused_combine=$fc"; grep -v '^{' $OUT/llm_bench_fc$fc.log | grep -E "decode|prefill"
done
