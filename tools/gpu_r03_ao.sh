#!/bin/bash
# Round 3 session AO: argmax with 8 loads in flight per thread (was 17.6 us in the T=1 step);
# overlap probe (can a forked consumer kernel wait on its producer inside a HIP graph?).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ao
mkdir -p $OUT
timeout -k 10 60 ./tools/debug/overlap_probe > $OUT/overlap_probe.log 2>&1; rc=$?
cat $OUT/overlap_probe.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_llm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "argmax or greedy or batched" > $OUT/pytest_llm.log 2>&1 || { tail -40 $OUT/pytest_llm.log; exit 1; }
tail -1 $OUT/pytest_llm.log
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t1 -o llm -- \
  python3 tools/steady_prof.py llm-decode --tokens 1 --iters 64 --warmup 8 > $OUT/prof_t1.log 2>&1 \
  || { tail -20 $OUT/prof_t1.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_t1 -name '*.db' | head -1) --after-gap-ms 200 \
  --per 64 --top 30 > $OUT/llm_decode_t1_kernels.txt && grep -E "argmax|busy" $OUT/llm_decode_t1_kernels.txt | cut -c1-150
