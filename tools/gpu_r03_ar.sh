#!/bin/bash
# Round 3 session AR: rehearsal of the tree after the in-graph argmax and the Q4_K ffn_down shape
# (long-row stages + 16 rows per workgroup at T = 1) — every GPU test, smoke(), bench.py, LLM
# decode / prefill, T = 1 and T = 4 steady-state kernel profiles.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ar
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-300
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
for T in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t$T -o llm -- \
    python3 tools/steady_prof.py llm-decode --tokens $T --iters 64 --warmup 8 > $OUT/prof_t$T.log 2>&1 \
    || { tail -20 $OUT/prof_t$T.log; exit 1; }
  python3 tools/rocpd_summary.py $(find $OUT/prof_t$T -name '*.db' | head -1) --after-gap-ms 200 \
    --per 64 --top 30 > $OUT/llm_decode_t${T}_kernels.txt && head -1 $OUT/llm_decode_t${T}_kernels.txt
done
