#!/bin/bash
# Round 3 session AM: round-end rehearsal of the final tree — every GPU test, smoke(), bench.py,
# LLM decode / prefill — plus the single-launch GroupNorm size gate at 128 KB vs the 64 KB default.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/am
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-300
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
for kb in 64 128; do
  AMDK8S_GN_FUSED_KB=$kb timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 \
    --miopen-find --out $OUT/sd15_bench_kb$kb.json > $OUT/sd15_bench_kb$kb.log 2>&1 || { tail -20 $OUT/sd15_bench_kb$kb.log; exit 1; }
  echo "AMDK8S_GN_FUSED_KB=$kb"; grep -E "unet|e2e" $OUT/sd15_bench_kb$kb.log
done
