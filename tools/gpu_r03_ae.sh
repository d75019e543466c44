#!/bin/bash
# Round 3 session AE: round-end rehearsal of the tree after the prefill / norm changes (every GPU
# test, smoke(), bench.py) + T=1 steady-state decode profile of the defaults.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ae
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t1 -o llm -- \
  python3 tools/steady_prof.py llm-decode --tokens 1 --iters 64 --warmup 8 > $OUT/prof_t1.log 2>&1 \
  || { tail -20 $OUT/prof_t1.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_t1 -name '*.db' | head -1) --after-gap-ms 200 \
  --per 64 --top 30 > $OUT/llm_decode_t1_kernels.txt && head -14 $OUT/llm_decode_t1_kernels.txt | cut -c1-150
