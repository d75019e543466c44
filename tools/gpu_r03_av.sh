#!/bin/bash
# Round 3 session AV: final rehearsal of the round's tree — every GPU test, smoke(), bench.py, LLM
# decode / prefill, steady-state prefill kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/av
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
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_prefill -o llm -- \
  python3 tools/steady_prof.py llm-prefill --iters 10 --warmup 3 > $OUT/prof_prefill.log 2>&1 \
  || { tail -20 $OUT/prof_prefill.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_prefill -name '*.db' | head -1) --after-gap-ms 200 \
  --per 10 --top 30 > $OUT/llm_prefill_kernels.txt && head -16 $OUT/llm_prefill_kernels.txt | cut -c1-170
