#!/bin/bash
# Round 3 session X: where the extra time of a T=4 decode step goes — steady-state kernel profile
# at T=4 (position 512..) with the session-W defaults, and per-shape GEMV / small-kernel timings
# at T=1 and T=4 (tools/llm_bench.py --gemv --kernels).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/x
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t4 -o llm -- \
  python3 tools/steady_prof.py llm-decode --tokens 4 --iters 64 --warmup 8 > $OUT/prof_t4.log 2>&1 \
  || { tail -20 $OUT/prof_t4.log; exit 1; }
tail -1 $OUT/prof_t4.log
python3 tools/rocpd_summary.py $(find $OUT/prof_t4 -name '*.db' | head -1) --after-gap-ms 200 \
  --per 64 --top 30 > $OUT/llm_decode_t4_kernels.txt && head -16 $OUT/llm_decode_t4_kernels.txt | cut -c1-150
timeout -k 10 500 python -u tools/llm_bench.py --tokens 1,4 --gemv --kernels --out $OUT/llm_bench.json \
  > $OUT/llm_bench.log 2>&1 || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|'gemv'|kernel" $OUT/llm_bench.log | cut -c1-200
