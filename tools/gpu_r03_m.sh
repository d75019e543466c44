#!/bin/bash
# Round 3 session M: LLM decode, register-resident activations for T = 3, 4 (AMDK8S_LLM_REGX_T A/B)
# on top of the once-per-input Q8 pass; tests with the new default.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/m
mkdir -p $OUT
for r in 2 4; do
  AMDK8S_LLM_REGX_T=$r timeout -k 10 400 python -u tools/llm_bench.py --gemv --out $OUT/llm_bench_regx$r.json \
    > $OUT/llm_bench_regx$r.log 2>&1 || { tail -30 $OUT/llm_bench_regx$r.log; exit 1; }
  echo "regx_t=$r"; grep -v '^{' $OUT/llm_bench_regx$r.log | grep -E "decode|prefill"
done
AMDK8S_LLM_REGX_T=4 timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_sd15_gpu.py > $OUT/pytest_sd15.log 2>&1 || { tail -40 $OUT/pytest_sd15.log; exit 1; }
tail -2 $OUT/pytest_sd15.log
timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
  --out $OUT/sd15_bench.json > $OUT/sd15_bench.log 2>&1 || { tail -20 $OUT/sd15_bench.log; exit 1; }
grep -E "unet|e2e" $OUT/sd15_bench.log
AMDK8S_GEMM_SPLITK=1 timeout -k 10 400 python -u tools/sd15_bench.py --arms native-graph --batches "" --miopen-find \
  --out $OUT/sd15_bench_nosplit.json > $OUT/sd15_bench_nosplit.log 2>&1 || { tail -20 $OUT/sd15_bench_nosplit.log; exit 1; }
echo "no split-K:"; grep -E "unet" $OUT/sd15_bench_nosplit.log
AMDK8S_GN_CHUNKS=64 timeout -k 10 400 python -u tools/sd15_bench.py --arms native-graph --batches "" --miopen-find \
  --out $OUT/sd15_bench_gn64.json > $OUT/sd15_bench_gn64.log 2>&1 || { tail -20 $OUT/sd15_bench_gn64.log; exit 1; }
echo "GN 64 chunks:"; grep -E "unet" $OUT/sd15_bench_gn64.log
