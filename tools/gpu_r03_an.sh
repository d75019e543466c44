#!/bin/bash
# Round 3 session AN: greedy argmax inside the decode step's HIP graph (Engine.decode_greedy, used
# by the server and the bench) — LLM GPU tests, decode T=1..4, T=1 steady-state profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/an
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t1 -o llm -- \
  python3 tools/steady_prof.py llm-decode --tokens 1 --iters 64 --warmup 8 > $OUT/prof_t1.log 2>&1 \
  || { tail -20 $OUT/prof_t1.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_t1 -name '*.db' | head -1) --after-gap-ms 200 \
  --per 64 --top 30 > $OUT/llm_decode_t1_kernels.txt && head -16 $OUT/llm_decode_t1_kernels.txt | cut -c1-150
